"""cProfile of the host side of graph-mode training steps (bench.py's flagship config).

    python tools/host_profile.py [bench.py flags]
"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    import bench
    import ewdml
    from ewdml.runtime.trainer import Trainer

    a = bench.parse(sys.argv[1:])
    levels = a.qsgd_levels or (127 if a.qsgd_bits == 8 else 7)
    flags = ["--network", a.network, "--dataset", a.dataset, "--batch-size", str(a.batch_size),
             "--compress", a.compress, "--topk-ratio", str(a.topk_ratio), "--qsgd-bits",
             str(a.qsgd_bits), "--qsgd-levels", str(levels), "--momentum", "0.9",
             "--bucket-mb", str(a.bucket_mb), "--synthetic-size", "16384", "--eval-freq", "0",
             "--quiet", "--hip-graph", a.hip_graph, "--graph-warmup", "2"]
    tr = Trainer(ewdml.parse_args(flags))
    for _ in range(6):
        tr.train_step()
    torch.cuda.synchronize()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(200):
        tr.train_step()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(25)
    print(s.getvalue())


if __name__ == "__main__":
    main()
