"""Host cost of replaying a HIP graph vs its node count (is a step launch-bound?).

    python tools/graph_launch_cost.py
Prints, for graphs of N tiny kernels, the host time of ``replay()`` (enqueue only) and the
end-to-end time per replay with the GPU draining.
"""
import time

import torch


def main():
    x = torch.zeros(1024, device="cuda")
    s = torch.cuda.Stream()
    for n in (10, 50, 150, 300):
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(3):
                x.add_(1.0)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for _ in range(n):
                    x.add_(1.0)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for _ in range(5):
            g.replay()
        torch.cuda.synchronize()
        reps = 50
        t0 = time.perf_counter()
        for _ in range(reps):
            g.replay()
        t1 = time.perf_counter()
        torch.cuda.synchronize()
        t2 = time.perf_counter()
        print(f"nodes={n:4d}  host enqueue/replay {1e6 * (t1 - t0) / reps:8.1f} us   "
              f"wall/replay {1e6 * (t2 - t0) / reps:8.1f} us   "
              f"per node {1e6 * (t2 - t0) / reps / n:6.2f} us")


if __name__ == "__main__":
    main()
