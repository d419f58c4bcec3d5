"""tools/cluster.py: the reference EC2 tool's host files and run/kill surface (CPU, local host)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tools"))

import cluster  # noqa: E402


def test_host_files(tmp_path):
    aliases = cluster.write_hosts(["10.0.0.5", "10.0.0.6"], str(tmp_path), ssh_user="me")
    assert aliases == ["ewdml-node1", "ewdml-node2"]
    assert (tmp_path / "hosts").read_text() == "10.0.0.5\tewdml-node1\n10.0.0.6\tewdml-node2\n"
    assert (tmp_path / "hosts_alias").read_text().split() == aliases
    assert cluster.read_hosts(str(tmp_path / "hosts")) == ["10.0.0.5", "10.0.0.6"]
    assert cluster.read_hosts(str(tmp_path / "hosts_address")) == ["10.0.0.5", "10.0.0.6"]
    cfg = (tmp_path / "ssh_config").read_text()
    assert "Host ewdml-node2\n\tHostName 10.0.0.6" in cfg and "User me" in cfg


def test_dry_run_commands(tmp_path, capsys):
    hf = tmp_path / "hosts_address"
    hf.write_text("10.0.0.1\n10.0.0.2\n")
    for cmd in ("sync", "status", "kill"):
        assert cluster.main([cmd, "--hosts", str(hf), "--workdir", "/w", "--dry-run"]) == 0
    assert cluster.main(["run", "--hosts", str(hf), "--workdir", "/w", "--gpus-per-node", "8",
                         "--dry-run", "--", "--network", "VGG11"]) == 0
    out = capsys.readouterr().out
    assert "rsync -az --delete" in out and "10.0.0.2:/w/" in out
    assert "--node-rank 1" in out and "--master-addr 10.0.0.1" in out and "setsid" in out
    assert "kill -TERM -- -$(cat .ewdml_run.pgid)" in out


def test_local_run_status_kill(tmp_path):
    hf = tmp_path / "hosts_address"
    hf.write_text("127.0.0.1\n")
    (tmp_path / "sleeper.py").write_text("import time\ntime.sleep(120)\n")
    logs = str(tmp_path / "logs")
    common = ["--hosts", str(hf), "--workdir", str(tmp_path), "--logdir", logs]
    assert cluster.main(["exec", *common, "--", "echo", "node-ok"]) == 0
    assert "node-ok" in open(os.path.join(logs, "exec_0.log")).read()
    # run blocks until the job ends: start it in the background through dispatch's Popen
    import subprocess

    run = subprocess.Popen([sys.executable, os.path.join(ROOT, "tools", "cluster.py"), "run",
                            *common, "--gpus-per-node", "1", "--master-port", "29621",
                            "--script", "sleeper.py"])
    try:
        state = ""
        for _ in range(60):
            assert cluster.main(["status", *common]) == 0
            state = open(os.path.join(logs, "status_0.log")).read()
            if "running" in state:
                break
            time.sleep(0.5)
        assert "running" in state
        assert cluster.main(["kill", *common]) == 0
        run.wait(timeout=60)
        assert cluster.main(["status", *common]) == 0
        assert "idle" in open(os.path.join(logs, "status_0.log")).read()
    finally:
        if run.poll() is None:
            run.kill()
