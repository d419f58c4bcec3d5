"""Spawn a CPU/Gloo world on 127.0.0.1 and collect per-rank results (reference test pattern:
``run_pytorch_single.sh`` -- several ranks on one host over Gloo)."""
import os
import socket
import traceback

import torch
import torch.multiprocessing as mp


def free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _entry(rank, world, port, fn, args, out_dir):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    import torch.distributed as dist
    try:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        res = fn(rank, world, *args)
        torch.save(res, os.path.join(out_dir, f"r{rank}.pt"))
    except BaseException:
        with open(os.path.join(out_dir, f"r{rank}.err"), "w") as f:
            f.write(traceback.format_exc())
        raise
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def run_world(fn, world, tmp_path, args=(), expect_fail=False):
    port = free_port()
    os.makedirs(str(tmp_path), exist_ok=True)
    out = str(tmp_path)
    ctx = mp.start_processes(_entry, args=(world, port, fn, args, out), nprocs=world,
                             join=False, start_method="spawn")
    try:
        while not ctx.join(timeout=120):
            pass
    except Exception as e:  # a rank failed
        if not expect_fail:
            errs = [open(os.path.join(out, f)).read() for f in os.listdir(out)
                    if f.endswith(".err")]
            raise AssertionError("\n".join(errs) or str(e))
        return None
    if expect_fail:
        raise AssertionError("expected a failure")
    return [torch.load(os.path.join(out, f"r{r}.pt"), weights_only=False) for r in range(world)]
