"""Per-kernel cost of back-to-back kernels in a replayed HIP graph: N tiny elementwise launches
(1 block, 256 blocks, 2048 blocks of trivial work) captured in one graph, us per kernel over 50
replays.  Separates the runtime / command-processor floor from a kernel's own latency chain."""
import torch

s = torch.cuda.Stream()
for blocks in (1, 256, 2048):
    x = torch.zeros(blocks * 256 * 4, device="cuda")
    n = 200
    with torch.cuda.stream(s):
        for _ in range(3):
            x.add_(1.0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(20):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    print(f"{blocks:5d} blocks: {a.elapsed_time(b) * 1e3 / (20 * n):6.2f} us per kernel", flush=True)

# Per-replay cost of a graph launch: the same 2 x 80 kernels as one graph of 160 replayed 20 times
# or a graph of 80 replayed 40 times (the difference over 20 launches is one launch boundary each).
x = torch.zeros(256 * 256 * 4, device="cuda")
res = {}
for n, reps in ((80, 40), (160, 20)):
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(n):
            x.add_(1.0)
    g.replay()
    torch.cuda.synchronize()
    best = 1e30
    for _ in range(5):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            g.replay()
        b.record()
        torch.cuda.synchronize()
        best = min(best, a.elapsed_time(b) * 1e3)
    res[n] = best
    print(f"graph of {n} kernels x {reps} replays: {best:8.1f} us", flush=True)
print(f"per graph-launch boundary: {(res[80] - res[160]) / 20:6.2f} us", flush=True)
