"""Flagship benchmark: VGG-11(-BN) on CIFAR-10-shaped synthetic data, top-1 % + 8-bit QSGD
gradient exchange with error feedback over RCCL, one process per MI355X, fp32 (the reference's
precision).

    python bench.py --gpus 1 --steps 50 --warmup 10
    python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 \
        --master-port 29500 bench.py --gpus 8 --steps 50 --warmup 10

Metric (BASELINE.json): "grad bytes/step on wire + images/sec, VGG-11 CIFAR-10 at 1/2/4/8
MI355X".  ``value`` = whole-job images/sec (sum over ranks: N x per-GPU batch x K / max-over-ranks
time of the K timed steps).  Every timed step is a full training step: on-device batch gather +
augmentation, fp32 forward/backward on the hand-written fp32 MFMA kernels (the reference trains in
fp32: ``src/distributed_worker.py:249-251``, ``src/optim/sgd.py:59-91``), per-bucket top-k + QSGD
encode with error feedback (HIP), RCCL all-gather of the packed payloads, fused decode + average +
SGD (HIP).  Weak scaling: the per-GPU batch is fixed as N grows.  The byte fields report the
payload per rank, the algorithmic wire bytes, and the reference-equivalent MiB/step.

Extra measured fields (same K / W, after the headline run): ``value_fp32_no_ef`` (the same step
without error feedback: its cost) and ``value_bf16`` / ``ms_per_step_bf16`` (bf16 autocast with bf16
weight copies, error feedback on).  ``--no-extras`` skips them.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

# The reference publishes no images/sec; BASELINE.md derives ~104 img/s aggregate for VGG-11 on
# its 2-worker Colab CPU setup from the end-to-end training-time chart.
BASELINE_IMG_S = 104.0


# BASELINE.json configs (the default is the headline VGG-11 one)
PRESETS = {
    "vgg11": dict(network="VGG11", dataset="Cifar10", topk_ratio=0.01, qsgd_bits=8),
    "lenet": dict(network="LeNet", dataset="MNIST", topk_ratio=0.01, qsgd_bits=8,
                  batch_size=64),
    "resnet50_cifar": dict(network="ResNet50", dataset="Cifar10", topk_ratio=0.01, qsgd_bits=8),
    "resnet50_imagenet": dict(network="resnet50_imagenet", dataset="imagenet", topk_ratio=0.001,
                              qsgd_bits=4, batch_size=64),
}


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--preset", default="vgg11", choices=sorted(PRESETS),
                   help="BASELINE.json config (explicit flags override it)")
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=32)
    p.add_argument("--warmup", type=int, default=8)
    p.add_argument("--network", default=None)
    p.add_argument("--dataset", default=None)
    p.add_argument("--batch-size", type=int, default=None, help="per-GPU batch (default 128)")
    p.add_argument("--compress", default="topk_qsgd")
    p.add_argument("--topk-ratio", type=float, default=None)
    p.add_argument("--qsgd-bits", type=int, default=None)
    p.add_argument("--qsgd-levels", type=int, default=None)
    p.add_argument("--bucket-mb", type=float, default=64.0)
    p.add_argument("--amp", default="none", help="none = fp32 (reference precision), bf16")
    p.add_argument("--channels-last", action="store_true")
    p.add_argument("--layout", default="auto", choices=["auto", "nchw", "nhwc"])
    p.add_argument("--fused-nn", default="on", choices=["on", "off"])
    p.add_argument("--no-overlap", action="store_true")
    p.add_argument("--error-feedback", default="on", choices=["on", "off"])
    p.add_argument("--no-extras", action="store_true", help="headline run only")
    # auto: the one-graph step at N = 1 and for top-k payloads; per-bucket collectives overlapped
    # with backward (segmented graphs) for large dense collectives at N > 1 (plan_graph_mode)
    p.add_argument("--hip-graph", default="auto",
                   choices=["auto", "off", "split", "full", "segmented"])
    # most steps per graph launch in the timed loop (Trainer.train_steps; the U <= this that needs
    # the fewest launches for --steps): the same steps, one launch boundary (~7.7 us,
    # tools/probes/launch_floor.py) per U steps; 1 = one graph per step.  16 vs 8: VGG-11 1.1401 /
    # 1.1408 vs 1.1454 / 1.1470 ms (profiles/ab/README.md)
    p.add_argument("--graph-unroll", type=int, default=16)
    p.add_argument("--param-dtype", default="auto", choices=["auto", "fp32"])
    p.add_argument("--json-out", default=None, help="also write the JSON line to this file")
    p.add_argument("--extra", default="", help="extra distributed_nn.py flags")
    a = p.parse_args(argv)
    pre = {"batch_size": 128, **PRESETS[a.preset]}
    for k, v in pre.items():
        if getattr(a, k) is None:
            setattr(a, k, v)
    return a


def _flags(a, world, amp, ef):
    levels = a.qsgd_levels or (127 if a.qsgd_bits == 8 else 7)
    flags = ["--network", a.network, "--dataset", a.dataset, "--batch-size", str(a.batch_size),
             "--compress", a.compress, "--topk-ratio", str(a.topk_ratio), "--qsgd-bits",
             str(a.qsgd_bits), "--qsgd-levels", str(levels), "--momentum", "0.9", "--lr", "0.01",
             "--bucket-mb", str(a.bucket_mb), "--amp", amp, "--synthetic-size",
             str(max(16384, 4 * a.batch_size * world)),
             "--eval-freq", "0", "--log-interval", "1000000", "--quiet",
             "--max-steps", str(a.steps + a.warmup)]
    if a.channels_last:
        flags.append("--channels-last")
    flags += ["--layout", a.layout, "--fused-nn", a.fused_nn]
    if a.no_overlap:
        flags.append("--no-overlap")
    if ef:  # the timed steps run the steady-state codec: no density / lr warm-up phase
        flags += ["--error-feedback", "--ef-warmup", "none"]
    else:
        flags.append("--no-error-feedback")
    # graph capture happens inside the untimed warmup: eager steps, then the capturing step
    gw = max(1, min(3, a.warmup - 1))
    flags += ["--hip-graph", a.hip_graph, "--graph-warmup", str(gw), "--param-dtype",
              a.param_dtype if amp != "none" else "fp32"]
    return flags + a.extra.split(), gw


def measure(a, world, amp, ef, extra=()):
    """Build a Trainer for this configuration, run W untimed warmup steps, then time exactly K
    steps bracketed by barrier + synchronize on both sides; returns (max-over-ranks seconds,
    trainer, final loss, host enqueue seconds, per-rank seconds [min, max], replica check).

    After the timed steps every rank fingerprints its flat parameters (fp64 sums and the XOR of
    the raw words) and all ranks compare them: synchronous data parallelism must leave the
    replicas bitwise identical, so a wrong collective on a first multi-GPU run shows up here
    instead of as a plausible img/s (local SGD's replicas legitimately differ between syncs:
    no check there)."""
    import torch

    import ewdml
    from ewdml.runtime.trainer import Trainer

    flags, gw = _flags(a, world, amp, ef)
    tr = Trainer(ewdml.parse_args(flags + list(extra), prog="bench.py"))
    try:
        return _measure(a, tr, gw)
    finally:
        tr.close()  # watchdog and own RCCL communicator (the next measure() builds its own)


def _any_rank(flag: bool) -> bool:
    """Whether ``flag`` holds on any rank (process-group all-reduce; every rank must call it)."""
    import torch
    import torch.distributed as dist

    if not dist.is_initialized() or dist.get_world_size() == 1:
        return bool(flag)
    dev = "cuda" if torch.cuda.is_available() and dist.get_backend() == "nccl" else "cpu"
    t = torch.tensor([1.0 if flag else 0.0], device=dev)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return bool(t.item() > 0)


def _pick_unroll(steps: int, umax: int) -> int:
    """Steps per graph launch for ``steps`` timed steps: the U <= umax that needs the fewest
    launches (K // U replays of the U-step graph + K % U one-step replays), the larger U on a tie;
    1 = one graph per step."""
    best = (steps, 1)
    for u in range(2, min(umax, steps) + 1):
        n = steps // u + steps % u
        if n < best[0] or (n == best[0] and u > best[1]):
            best = (n, u)
    return best[1]


def _measure(a, tr, gw):
    import torch

    def sync():
        if tr.cuda:
            torch.cuda.synchronize()

    warm = a.warmup if a.hip_graph == "off" else max(a.warmup, gw + 1)
    every = getattr(tr.exchange, "every", 1)
    if a.hip_graph != "off" and every > 1:
        # local SGD captures two steps (local, sync): both before the clock starts
        warm = max(warm, every + gw)
    # --graph-unroll U (when the timed run holds at least one run of U steps): the U-step graph is
    # captured and replayed once as the last U warmup steps (at least gw + 1 one-step warmup steps
    # before it: the eager steps and the one-step capture)
    unroll = _pick_unroll(a.steps, a.graph_unroll)
    single = warm if unroll == 1 else max(gw + 1, warm - unroll)
    for _ in range(single):
        tr.train_step()
    if unroll > 1 and tr.prepare_unrolled(unroll):
        tr.train_steps(unroll, unroll)
    else:
        for _ in range(warm - single):
            tr.train_step()
        unroll = 1
    tr.graph_unroll_used = unroll
    tr.warmup_run = single + (unroll if unroll > 1 else warm - single)
    sync()
    tr.comm.barrier()
    sync()
    if os.environ.get("EWDML_PROF_GAP") == "1":  # idle gap marking the timed region in traces
        time.sleep(0.25)
    t0 = time.perf_counter()
    loss = None
    loss, _ = tr.train_steps(a.steps, unroll)
    t_enq = time.perf_counter()  # host done enqueuing (the GPU may still be running)
    sync()
    t1 = time.perf_counter()
    if os.environ.get("EWDML_PROF_GAP") == "1":  # ... and after it (outside the clock)
        time.sleep(0.25)
    tr.comm.barrier()
    sync()
    elapsed_max = tr.comm.all_reduce_scalars([t1 - t0], op="max")[0]
    elapsed_min = -tr.comm.all_reduce_scalars([-(t1 - t0)], op="max")[0]
    from ewdml.parallel.engine import check_replicas

    ge = getattr(tr.exchange, "inner", tr.exchange)
    # top-k encode counters; raises if a write block gave up on its look-back (corrupt payload).
    # The counters are per rank: the verdict is agreed after the replica check (which every rank
    # must reach), so all ranks raise together and stay in step for the next measurement.
    health_err = None
    try:
        tr.codec_health = ge.codec_health() if hasattr(ge, "codec_health") else {}
    except Exception as exc:  # noqa: BLE001
        health_err = repr(exc)
        tr.codec_health = {"error": health_err[:300]}

    rep = None if every > 1 else check_replicas(tr.comm, tr.flat.data)
    if _any_rank(health_err is not None):
        raise RuntimeError(f"codec health check failed on some rank: {health_err}")
    final_loss = float(loss.detach()) if loss is not None else float("nan")
    tr.comm_kind = tr.comm.kind
    tr.comm_probe = None if tr.comm.probe is None else {
        k: tr.comm.probe[k] for k in ("ok", "eager", "graph")}
    g = getattr(tr, "_graphs", None)
    tr.overlap_comm_graphs = len(g[1].comms) if (g and g[0] == "segmented") else 0
    return elapsed_max, tr, final_loss, t_enq - t0, (elapsed_min, elapsed_max), rep


def main(argv=None):
    a = parse(argv)
    import torch
    import torch.distributed as dist

    import ewdml
    from ewdml.utils.metrics import byte_summary

    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus:
        raise SystemExit(f"--gpus {a.gpus} but WORLD_SIZE={world}; launch with torch.distributed.run")
    ef = a.error_feedback == "on"
    elapsed_max, tr, final_loss, enq, span, rep = measure(a, world, a.amp, ef)
    cuda = tr.cuda
    ms = elapsed_max * 1e3 / a.steps
    img_s = world * a.batch_size * a.steps / elapsed_max
    bytes_ = byte_summary(tr.exchange.last, world)
    metric = "grad bytes/step on wire + images/sec, VGG-11 CIFAR-10 at 1/2/4/8 MI355X"
    if a.preset != "vgg11":
        metric = f"grad bytes/step on wire + images/sec, {a.network} {a.dataset}"
    nb = len(tr.flat.buckets)
    rec = {
        "metric": metric,
        "value": round(img_s, 2),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        # untimed steps actually run (>= warmup: the eager steps before the graph capture and, with
        # --graph-unroll, one replay of the U-step graph)
        "warmup_steps_run": getattr(tr, "warmup_run", a.warmup),
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(img_s / BASELINE_IMG_S, 2) if a.preset == "vgg11" else None,
        "baseline_note": "reference publishes no img/s; BASELINE.md derives ~104 img/s (VGG-11, "
                         "2 Colab CPU workers)",
        # the compute dtype actually used (--amp bf16 on a model whose fused fp32 step is faster
        # -- LeNet -- trains in fp32: Trainer.amp_kept_fp32)
        "dtype": getattr(tr, "compute_dtype", a.amp if a.amp != "none" else "fp32"),
        "amp_requested": a.amp,
        "data": f"synthetic ({a.dataset} shape {'x'.join(map(str, tr.info['shape']))}, "
                f"{tr.info['classes']} classes, random-init weights)",
        "config": {"model": "vgg11_bn" if a.network.lower() in ("vgg11", "vgg11_bn") else
                   a.network, "global_batch": world * a.batch_size, "per_gpu_batch": a.batch_size,
                   "seq_len": None, "parallelism": f"dp{world}",
                   "codec": tr.exchange.codec.describe() if hasattr(tr.exchange, "codec") else
                   a.compress, "error_feedback": ef, "optimizer": "sgd(momentum=0.9)",
                   "overlap_requested": not a.no_overlap, "buckets": nb, "hip_graph": tr.graph_mode,
                   "bf16_params": tr.flat.shadow is not None,
                   "grad_mode": "views" if tr.flat.attach_grads else "pointers",
                   "layout": "nhwc" if tr.channels_last else "nchw",
                   "fused_nn": a.fused_nn, "comm": tr.comm_kind,
                   "local_apply": bool(getattr(getattr(tr.exchange, "inner", tr.exchange),
                                               "local_apply", False)),
                   "wgrad_stream": bool(getattr(tr, "wgrad_stream", False))},
        # overlap that actually happens: a collective to hide (world > 1) issued while backward
        # still runs -- a segmented graph with at least one comm-stream graph, or eager steps
        # with the side stream and more than one bucket
        "overlap_effective": bool(world > 1 and not a.no_overlap and (
            tr.overlap_comm_graphs > 0 or (tr.graph_mode == "off" and nb > 1))),
        "overlap_comm_graphs": tr.overlap_comm_graphs,
        "grad_bytes_per_step_on_wire": bytes_["wire_bytes_total"],
        "payload_bytes_per_rank": bytes_["payload_bytes_per_rank"],
        "dense_fp32_grad_bytes": bytes_["dense_fp32_bytes"],
        "compression_ratio": bytes_["compression_ratio"],
        "ref_equiv_MiB_per_step": round(bytes_["ref_equiv_MiB_per_step"], 4),
        "ref_equiv_reduction": bytes_["ref_equiv_reduction"],
        "final_loss": final_loss,
        # a throughput run, not a convergence one: W + K steps from random init with the
        # steady-state codec (no EF density / lr warm-up, which the CLI default --ef-warmup auto
        # runs); convergence with error feedback: profiles/validation/ef_stability_r03.md
        "final_loss_note": f"{a.warmup + a.steps} steps from random init, steady-state codec "
                           "without the EF warm-up (see profiles/validation/ef_stability_r03.md)",
        "host_enqueue_ms_per_step": round(enq * 1e3 / a.steps, 4),
        "graph_unroll": getattr(tr, "graph_unroll_used", 1),
        # multi-GPU self-validation: replicas bitwise identical after the timed steps, the
        # data-plane communicator and its first-contact probe (parallel/probe.py)
        # (None under local SGD between syncs: the replicas agree only right after a sync step)
        "replicas_identical": rep["identical"] if rep is not None else None,
        "replica_fingerprint": rep["fingerprints"][0] if rep is not None else None,
        "comm": tr.comm_kind,
        "rccl_world": world if tr.comm_kind == "rccl-stream" else 0,
        "comm_probe": tr.comm_probe,
        "graph_plan": tr.graph_plan,
        # the N > 1 step model's prediction for the mode that ran (parallel/step_model.py: N = 1
        # measurements + an xGMI collective model), to check a scaling run against
        "predicted_ms_per_step": ((tr.graph_plan or {}).get("predicted_ms") or {}).get(
            "segmented" if tr.graph_mode == "segmented" else "full"),
        # the step model against this run at N = 1, where it has no collective term to blame
        # (|error| <= 3 % on the committed preset lines: tests/unit/test_graph_plan.py)
        "model_error_n1": None,
        "codec_health": tr.codec_health,
        "step_ms_min": round(span[0] * 1e3 / a.steps, 4),
        "step_ms_max": round(span[1] * 1e3 / a.steps, 4),
        "hip_ext": ewdml.ops.library_path() if cuda else None,
    }
    if world == 1 and rec["predicted_ms_per_step"]:
        rec["model_error_n1"] = round(rec["predicted_ms_per_step"] / rec["ms_per_step"] - 1, 4)
    del tr
    if not a.no_extras:
        extras = []
        if ef:
            extras.append(("fp32_no_ef" if a.amp == "none" else f"{a.amp}_no_ef", a.amp, False,
                           ()))
        if a.amp == "none":
            extras.append(("bf16", "bf16", ef, ()))
            # the reference's live path (Method 3: dense fp32 gradients, all-reduce) and its
            # lowest-traffic one (Method 6: Method 5 + local SGD, sync every 20 steps)
            extras.append(("dense_fp32", "none", False, ("--compress", "none")))
            extras.append(("method6", "none", False, ("--method", "6")))
        for key, amp, e, xf in extras:
            if cuda:
                torch.cuda.empty_cache()
            err = None
            try:
                el, tr2, fl, _, _, rep2 = measure(a, world, amp, e, xf)
            except Exception as exc:  # noqa: BLE001 - an extra never costs the headline line
                err = repr(exc)[:300]
            # agreed by every rank before the next measurement's collectives (a failure on one
            # rank skips this extra everywhere)
            if _any_rank(err is not None):
                rec[f"error_{key}"] = err or "failed on another rank"
                continue
            if rep2 is not None:
                rec[f"replicas_identical_{key}"] = rep2["identical"]
            rec[f"value_{key}"] = round(world * a.batch_size * a.steps / el, 2)
            rec[f"dtype_{key}"] = getattr(tr2, "compute_dtype", amp)
            rec[f"ms_per_step_{key}"] = round(el * 1e3 / a.steps, 4)
            rec[f"final_loss_{key}"] = fl
            if key == "method6":
                ex = tr2.exchange
                rec["method6_sync_every"] = ex.every
                rec["method6_payload_bytes_per_sync"] = ex.bytes_per_step().payload_bytes
                rec["method6_hip_graph"] = tr2.graph_mode
            del tr2
    if dist.is_initialized():
        rank = dist.get_rank()
    else:
        rank = 0
    if rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    diverged = [k for k, v in rec.items() if k.startswith("replicas_identical") and v is False]
    if dist.is_initialized():
        dist.destroy_process_group()
    if diverged:  # every rank knows (the check is collective): fail the job loudly
        raise SystemExit(f"replicas differ after the timed steps ({', '.join(diverged)}): the "
                         "data-plane collectives are wrong; the img/s above is not valid")
    return rec


if __name__ == "__main__":
    main()
