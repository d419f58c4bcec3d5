"""Multi-node launcher: one ``torchrun`` per host over ssh (replaces the reference's EC2/pdsh
tooling, ``PS/tools/pytorch_ec2.py`` + ``src/launch.sh`` + ``src/run_pytorch_dist.sh``).

    python tools/launch.py --hosts hosts.txt --gpus-per-node 8 --workdir /path/to/repo -- \
        --network VGG11 --dataset Cifar10 --method 5 --batch-size 128 --max-steps 1000

``hosts.txt`` has one hostname/IP per line; the first is the rendezvous master.  Every node runs
``torchrun --nnodes N --node-rank i --nproc-per-node G --master-addr <host0> --master-port P
distributed_nn.py <args>`` (env:// rendezvous exactly like the reference's
``torch.distributed.launch`` scripts).  ``--dry-run`` prints the commands; ``--local`` runs the
single-node command here (``src/run_pytorch_single.sh`` equivalent).  Output of node i goes to
``<logdir>/node_i.log``; the launcher waits for all nodes and returns the worst exit code.
"""
import argparse
import os
import shlex
import subprocess
import sys


def build_commands(hosts, gpus, workdir, port, script, args, env=()):
    n = len(hosts)
    cmds = []
    for i, h in enumerate(hosts):
        envs = " ".join(f"{k}={shlex.quote(v)}" for k, v in env)
        cmd = (f"cd {shlex.quote(workdir)} && {envs} {sys.executable} -m torch.distributed.run "
               f"--nnodes {n} --node-rank {i} --nproc-per-node {gpus} --master-addr {hosts[0]} "
               f"--master-port {port} {script} " + " ".join(shlex.quote(a) for a in args))
        cmds.append((h, cmd.replace("  ", " ")))
    return cmds


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    if "--" in argv:
        k = argv.index("--")
        argv, train_args = argv[:k], argv[k + 1:]
    else:
        train_args = []
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--hosts", help="file with one host per line")
    ap.add_argument("--gpus-per-node", type=int, default=8)
    ap.add_argument("--workdir", default=os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    ap.add_argument("--master-port", type=int, default=29500)
    ap.add_argument("--script", default="distributed_nn.py")
    ap.add_argument("--logdir", default="launch_logs")
    ap.add_argument("--dry-run", action="store_true")
    ap.add_argument("--local", action="store_true", help="single node, run here")
    ap.add_argument("--ssh", default="ssh -o StrictHostKeyChecking=no")
    a = ap.parse_args(argv)
    env = [("HSA_ENABLE_IPC_MODE_LEGACY", "0")]
    hosts = ["127.0.0.1"] if a.local or not a.hosts else \
        [h.strip() for h in open(a.hosts) if h.strip() and not h.startswith("#")]
    cmds = build_commands(hosts, a.gpus_per_node, a.workdir, a.master_port, a.script, train_args,
                          env)
    if a.dry_run:
        for h, c in cmds:
            print(f"[{h}] {c}")
        return 0
    os.makedirs(a.logdir, exist_ok=True)
    procs = []
    for i, (h, c) in enumerate(cmds):
        log = open(os.path.join(a.logdir, f"node_{i}.log"), "w")
        full = ["bash", "-lc", c] if (a.local or h in ("127.0.0.1", "localhost")) else \
            shlex.split(a.ssh) + [h, c]
        procs.append((subprocess.Popen(full, stdout=log, stderr=subprocess.STDOUT), log))
    rc = 0
    for p, log in procs:
        rc = max(rc, p.wait())
        log.close()
    return rc


if __name__ == "__main__":
    sys.exit(main())
