"""Isolate HIP-graph capture failures: each case runs in its own subprocess."""
import subprocess
import sys

CASES = [
    ("lenet_none_split", ["--network", "LeNet", "--dataset", "MNIST", "--amp", "none", "--hip-graph", "split"]),
    ("lenet_none_full", ["--network", "LeNet", "--dataset", "MNIST", "--amp", "none", "--hip-graph", "full"]),
    ("lenet_bf16_split", ["--network", "LeNet", "--dataset", "MNIST", "--amp", "bf16", "--hip-graph", "split"]),
    ("lenet_bf16_full", ["--network", "LeNet", "--dataset", "MNIST", "--amp", "bf16", "--hip-graph", "full"]),
    ("vgg_none_full", ["--network", "VGG11", "--dataset", "Cifar10", "--amp", "none", "--hip-graph", "full"]),
    ("lenet_none_full_nooverlap", ["--network", "LeNet", "--dataset", "MNIST", "--amp", "none", "--hip-graph", "full", "--no-overlap"]),
    ("lenet_none_full_relaxed", ["--network", "LeNet", "--dataset", "MNIST", "--amp", "none", "--hip-graph", "full"], {"EWDML_GRAPH_CAPTURE_MODE": "relaxed"}),
]
BASE = ["--batch-size", "32", "--synthetic-size", "1024", "--momentum", "0.9", "--eval-freq", "0",
        "--quiet", "--device", "cuda", "--graph-warmup", "2", "--max-steps", "6",
        "--log-interval", "3"]

if __name__ == "__main__":
    import os
    for case in CASES:
        name, flags = case[0], case[1]
        env = dict(os.environ, **(case[2] if len(case) > 2 else {}))
        r = subprocess.run([sys.executable, "-X", "faulthandler", "distributed_nn.py"] + BASE + flags,
                           capture_output=True, text=True, timeout=300, env=env)
        lines = (r.stdout + r.stderr).strip().splitlines()
        tail = lines[-4:] if r.returncode == 0 else [l for l in lines if "File" in l][:8]
        print(f"== {name}: rc={r.returncode}")
        for t in tail:
            print("   ", t[:200])
        sys.stdout.flush()
