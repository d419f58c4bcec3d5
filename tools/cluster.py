"""Cluster housekeeping for multi-node runs: the command surface of the reference's EC2 tool
(``PyTorch-parameter-server/tools/pytorch_ec2.py`` ``get_hosts`` / ``run_command`` /
``kill_python`` / ``clean_launch_and_run``, ``tools/update_git_dir.sh``, ``tools/killall.sh``,
``tools/pre_run.sh``) for machines that already exist -- provisioning cloud instances (boto3 spot
requests) is out of scope: MI355X nodes are not rented per run through this tool.

    python tools/cluster.py hosts 10.0.0.1 10.0.0.2 ...   # writes hosts, hosts_address,
                                                           # hosts_alias, ssh_config
    python tools/cluster.py exec  --hosts hosts_address -- 'rocm-smi --showuse'
    python tools/cluster.py sync  --hosts hosts_address --workdir /path/to/repo
    python tools/cluster.py run   --hosts hosts_address --gpus-per-node 8 -- --network VGG11 ...
    python tools/cluster.py status --hosts hosts_address
    python tools/cluster.py kill  --hosts hosts_address

``run`` starts one ``torchrun`` per node (``tools/launch.py``'s commands) in a process group of its
own and records that group's id in ``<workdir>/.ewdml_run.pgid`` on the node; ``status`` and
``kill`` act on exactly that recorded group (never on processes matched by name, unlike the
reference's ``killall python``).  Every subcommand takes ``--dry-run`` (print the per-host commands)
and writes per-host output to ``<logdir>/<subcommand>_<i>.log``.
"""
import argparse
import os
import shlex
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from launch import build_commands  # noqa: E402

PGID_FILE = ".ewdml_run.pgid"


def read_hosts(path):
    """Addresses from a ``hosts_address`` file (one per line) or a ``hosts`` file (address and
    alias per line); ``#`` comments and blank lines skipped."""
    out = []
    with open(path) as f:
        for line in f:
            line = line.split("#", 1)[0].strip()
            if line:
                out.append(line.split()[0])
    return out


def write_hosts(addrs, outdir=".", alias_prefix="ewdml-node", ssh_user=None):
    """The reference's ``get_hosts`` outputs: ``hosts`` (``addr<TAB>alias``, rank order: the
    first is the rendezvous master), ``hosts_address``, ``hosts_alias``, and an ssh client config
    mapping each alias to its address (the reference's ``tools/config``)."""
    os.makedirs(outdir, exist_ok=True)
    aliases = [f"{alias_prefix}{i + 1}" for i in range(len(addrs))]
    with open(os.path.join(outdir, "hosts"), "w") as f:
        f.writelines(f"{a}\t{n}\n" for a, n in zip(addrs, aliases))
    with open(os.path.join(outdir, "hosts_address"), "w") as f:
        f.writelines(f"{a}\n" for a in addrs)
    with open(os.path.join(outdir, "hosts_alias"), "w") as f:
        f.writelines(f"{n}\n" for n in aliases)
    with open(os.path.join(outdir, "ssh_config"), "w") as f:
        for a, n in zip(addrs, aliases):
            f.write(f"Host {n}\n\tHostName {a}\n\tStrictHostKeyChecking no\n")
            if ssh_user:
                f.write(f"\tUser {ssh_user}\n")
    return aliases


def _wd(workdir):
    return shlex.quote(workdir)


def exec_commands(hosts, command):
    return [(h, command) for h in hosts]


def sync_commands(hosts, workdir, src):
    """rsync of the local tree to every host (``update_git_dir.sh``: the reference pulled git on
    each worker); build outputs travel too, results and logs do not."""
    excl = " ".join(f"--exclude {shlex.quote(e)}" for e in
                    (".git/", "gpurun_out/", "launch_logs/", "output/", "*.log", "__pycache__/"))
    return [(h, f"rsync -az --delete {excl} {shlex.quote(src.rstrip('/') + '/')} "
                f"{h}:{_wd(workdir)}/") for h in hosts]


def run_commands(hosts, gpus, workdir, port, script, args, env=()):
    """``tools/launch.py``'s torchrun per node, started with ``setsid`` so the node's whole job is
    one process group whose id is recorded for ``status`` / ``kill``."""
    out = []
    for h, cmd in build_commands(hosts, gpus, workdir, port, script, args, env):
        inner = f"echo $$ > {PGID_FILE} && exec bash -c {shlex.quote(cmd)}"
        out.append((h, f"cd {_wd(workdir)} && setsid bash -c {shlex.quote(inner)}"))
    return out


def status_commands(hosts, workdir):
    return [(h, f"cd {_wd(workdir)} && if [ -f {PGID_FILE} ] && kill -0 -- -$(cat {PGID_FILE}) "
                f"2>/dev/null; then echo running pgid=$(cat {PGID_FILE}); else echo idle; fi")
            for h in hosts]


def kill_commands(hosts, workdir, sig="TERM"):
    return [(h, f"cd {_wd(workdir)} && if [ -f {PGID_FILE} ]; then kill -{sig} -- "
                f"-$(cat {PGID_FILE}) 2>/dev/null; rm -f {PGID_FILE}; fi; echo done")
            for h in hosts]


def _is_local(h):
    return h in ("127.0.0.1", "localhost")


def dispatch(cmds, ssh, logdir, tag, local_only=False):
    """Run every (host, command) in parallel (rsync commands run here), wait, return the worst
    exit code; per-host output in ``<logdir>/<tag>_<i>.log``."""
    os.makedirs(logdir, exist_ok=True)
    procs = []
    for i, (h, c) in enumerate(cmds):
        log = open(os.path.join(logdir, f"{tag}_{i}.log"), "w")
        if local_only or _is_local(h) or c.startswith("rsync "):
            full = ["bash", "-c", c]
        else:
            full = shlex.split(ssh) + [h, c]
        procs.append((subprocess.Popen(full, stdout=log, stderr=subprocess.STDOUT), log))
    rc = 0
    for p, log in procs:
        rc = max(rc, p.wait())
        log.close()
    return rc


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    tail = []
    if "--" in argv:
        k = argv.index("--")
        argv, tail = argv[:k], argv[k + 1:]
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("cmd", choices=["hosts", "exec", "sync", "run", "status", "kill"])
    ap.add_argument("addrs", nargs="*", help="hosts: the node addresses, master first")
    ap.add_argument("--hosts", default="hosts_address", help="hosts / hosts_address file")
    ap.add_argument("--outdir", default=".", help="hosts: where the host files go")
    ap.add_argument("--ssh-user", default=None)
    ap.add_argument("--workdir", default=os.path.dirname(HERE))
    ap.add_argument("--src", default=os.path.dirname(HERE), help="sync: local tree to copy")
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--master-port", type=int, default=29500)
    ap.add_argument("--script", default="distributed_nn.py")
    ap.add_argument("--signal", default="TERM")
    ap.add_argument("--logdir", default="launch_logs")
    ap.add_argument("--ssh", default="ssh -o StrictHostKeyChecking=no")
    ap.add_argument("--dry-run", action="store_true")
    a = ap.parse_args(argv)
    if a.cmd == "hosts":
        if not a.addrs:
            ap.error("hosts needs the node addresses")
        for addr, alias in zip(a.addrs, write_hosts(a.addrs, a.outdir, ssh_user=a.ssh_user)):
            print(f"{addr}\t{alias}")
        return 0
    hosts = read_hosts(a.hosts)
    if a.cmd == "exec":
        if not tail:
            ap.error("exec needs a command after --")
        cmds = exec_commands(hosts, " ".join(tail))
    elif a.cmd == "sync":
        cmds = sync_commands(hosts, a.workdir, a.src)
    elif a.cmd == "run":
        cmds = run_commands(hosts, a.gpus_per_node, a.workdir, a.master_port, a.script, tail,
                            [("HSA_ENABLE_IPC_MODE_LEGACY", "0")])
    elif a.cmd == "status":
        cmds = status_commands(hosts, a.workdir)
    else:
        cmds = kill_commands(hosts, a.workdir, a.signal)
    if a.dry_run:
        for h, c in cmds:
            print(f"[{h}] {c}")
        return 0
    return dispatch(cmds, a.ssh, a.logdir, a.cmd)


if __name__ == "__main__":
    sys.exit(main())
