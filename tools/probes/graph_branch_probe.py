"""Do independent branches of a captured HIP graph run concurrently on this ROCm build?

Captures the same work (two chains of small bf16 GEMMs, each well below one chip's worth of
workgroups) once on a single stream and once forked over two streams (event fork/join), replays
both and prints the per-replay times.  If the two-stream graph is not faster, the runtime
serialises graph branches and side-stream overlap inside the step graph buys nothing.

    python tools/probes/graph_branch_probe.py
"""
import torch


def chain(a, b, n):
    for _ in range(n):
        a = a @ b
    return a


def capture(fn):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g, stream=s):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return g


def time_graph(g, reps=20):
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    n = 40
    for m in (256, 1024, 2048):
        a1 = torch.randn(m, 512, device="cuda", dtype=torch.bfloat16)
        a2 = torch.randn(m, 512, device="cuda", dtype=torch.bfloat16)
        b = torch.randn(512, 512, device="cuda", dtype=torch.bfloat16) / 23

        def serial():
            chain(a1, b, n)
            chain(a2, b, n)

        side = torch.cuda.Stream()

        def forked():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            chain(a1, b, n)
            with torch.cuda.stream(side):
                chain(a2, b, n)
            cur.wait_stream(side)

        def one():
            chain(a1, b, n)

        t1 = time_graph(capture(one))
        ts = time_graph(capture(serial))
        tf = time_graph(capture(forked))
        print(f"m={m:5d}  one chain {t1:8.1f} us   two serial {ts:8.1f} us   two forked {tf:8.1f} us"
              f"   forked/serial {tf / ts:.2f}", flush=True)


if __name__ == "__main__":
    main()
