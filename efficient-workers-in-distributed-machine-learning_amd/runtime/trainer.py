"""Training driver: one process per GPU, every rank a worker (or rank 0 a server with
``--topology ps``).

Parity: the roles of ``distributed_nn.py:123-146`` (rank dispatch), ``DistributedWorker.train_updated``
(``distributed_worker.py:162-239``: forward, backward, send grads, fetch grads, SGD step, accuracy,
log, periodic ``model_step_`` save) and ``SyncReplicasMaster_NN.start_updated``
(``sync_replicas_master_nn.py:158-177``).  Fixed defects: replicas start from rank 0's weights,
data is sharded with equal step counts on every rank, the loop ends on ``--max-steps`` *or*
``--epochs`` identically everywhere (no deadlock), only rank 0 checkpoints.
"""
import contextlib
import math
import os
import time

import torch
import torch.nn.functional as F

from ..compress.codecs import make_codec
from ..config import Config
from ..data import DeviceLoader, load_dataset
from ..models import build_model, canonical_name, input_shape
from ..models.fused import set_enabled as set_fused_nn
from ..optim.flat import make_optimizer
from ..parallel.comm import Comm, init_distributed
from ..parallel.engine import (GradientExchange, SegmentedCapture, StepStats, Stopwatch,
                               plan_graph_mode, sync_buffers, sync_params)
from ..parallel.flat import FlatModel
from ..parallel.local_sgd import LocalSGDExchange
from ..parallel.ps import PSExchange
from ..parallel.sharded import ShardedPSExchange
from ..utils import checkpoint as ckpt
from ..utils.metrics import MetricsLogger, accuracy, byte_summary

# full-step graph replays on the caller's stream (0: on the graph stream, with an event hop each
# way per step)
_SAME_STREAM_REPLAY = os.environ.get("EWDML_GRAPH_SAME_STREAM", "1") != "0"


def resolve_device(cfg: Config) -> torch.device:
    want = cfg.device
    if cfg.no_cuda:
        want = "cpu"
    if want == "auto":
        want = "cuda" if torch.cuda.is_available() else "cpu"
    if want == "cuda":
        local = int(os.environ.get("LOCAL_RANK", cfg.local_rank or 0))
        torch.cuda.set_device(local)
        return torch.device("cuda", local)
    return torch.device("cpu")


class FaultInjected(RuntimeError):
    pass


class Trainer:
    def __init__(self, cfg: Config, comm: Comm = None):
        self.cfg = cfg = cfg.resolved()
        self.device = resolve_device(cfg)
        # straggler mode 'kill' (distributed_nn.py:50-53) bounds only the per-step push
        # (parallel/ps.py k-of-n receive): setup, MIOpen find, graph capture, checkpoint and
        # eval collectives keep --comm-timeout
        timeout = cfg.comm_timeout
        self._own_comm = comm is None
        self.comm = comm or init_distributed(timeout_s=timeout,
                                             device=self.device if self.device.type == "cuda"
                                             else None)
        self.rank, self.world = self.comm.rank, self.comm.world
        self.cuda = self.device.type == "cuda"
        if cfg.sync_debug:
            from .. import ops
            ops.set_sync_debug(True)
            if cfg.hip_graph not in ("off", "auto"):
                raise ValueError("--sync-debug synchronises after each launch: use --hip-graph off")
        torch.manual_seed(cfg.seed)
        if self.cuda:
            from ..ops import head as _head

            _head.set_seed(cfg.seed, self.rank)  # dropout masks of the fused VGG head
        if self.cuda:  # MIOpen find once per shape during warmup (EWDML_CUDNN_BENCHMARK=0: heuristics)
            torch.backends.cudnn.benchmark = os.environ.get("EWDML_CUDNN_BENCHMARK", "1") == "1"
        self.log = MetricsLogger(cfg.metrics_file, self.rank, cfg.quiet)
        self.is_server = cfg.topology == "ps" and self.rank == 0

        # data -------------------------------------------------------------------------------
        net = canonical_name(cfg.network)
        set_fused_nn(cfg.fused_nn == "on")
        # activations channels_last where the fused NHWC conv-BN-ReLU-pool kernels run (VGG on the
        # GPU): MIOpen's convolutions are NHWC internally, so NCHW pays a transpose per conv
        self.channels_last = cfg.layout == "nhwc" or (
            cfg.layout == "auto" and self.cuda and cfg.fused_nn == "on"
            and net.startswith(("vgg", "resnet")))
        hold = int(cfg.holdout_from_test)
        x, y, info = load_dataset(cfg.dataset, cfg.data_dir, train=hold <= 0,
                                  synthetic_size=cfg.synthetic_size, seed=cfg.seed,
                                  device=self.device)
        if hold > 0:  # train / held-out split of the test set (only a test split on disk)
            if hold >= x.shape[0]:
                raise ValueError(f"--holdout-from-test {hold} >= {x.shape[0]} samples")
            tx, ty = x[-hold:], y[-hold:]
            x, y = x[:-hold], y[:-hold]
        if tuple(info["shape"]) != tuple(input_shape(net)):
            raise ValueError(f"{cfg.network} expects inputs {input_shape(net)}, dataset "
                             f"{cfg.dataset} has {info['shape']}")
        self.info = info
        n_workers = self.world - 1 if cfg.topology == "ps" else self.world
        w_rank = self.rank - 1 if cfg.topology == "ps" else self.rank
        # a model whose fused fp32 training step is faster than its bf16 autocast path (LeNet:
        # 0.10 vs 0.28 ms per step, latency-bound, ops/lenet.py) keeps that step under
        # --amp bf16: bf16 is a request for speed, and the fp32 step is also the more precise
        # one.  The compute dtype actually used is self.compute_dtype (bench.py reports it);
        # EWDML_AMP_FUSED_FP32=0: bf16 autocast anyway
        from ..models import fused_fp32_beats_amp

        self.amp_kept_fp32 = bool(self.cuda and cfg.amp == "bf16" and cfg.fused_nn == "on"
                                  and fused_fp32_beats_amp(net)
                                  and os.environ.get("EWDML_AMP_FUSED_FP32", "1") != "0")
        self.loader = None
        if not self.is_server:
            self.loader = DeviceLoader(x, y, info, cfg.batch_size, rank=w_rank,
                                       world=n_workers, shuffle=True,
                                       augment=cfg.augment and info["shape"][0] == 3,
                                       seed=cfg.seed, device=self.device,
                                       channels_last=self.channels_last,
                                       fused=self.cuda and cfg.fused_data == "on",
                                       out_dtype=torch.bfloat16 if (
                                           self.cuda and cfg.amp == "bf16"
                                           and not self.amp_kept_fp32) else torch.float32)
        if hold <= 0:
            tx, ty, _ = load_dataset(cfg.dataset, cfg.data_dir, train=False,
                                     synthetic_size=(cfg.synthetic_size // 5)
                                     if cfg.synthetic_size else 0,
                                     seed=cfg.seed, device=self.device)
        self.test_loader = DeviceLoader(tx, ty, info, min(cfg.test_batch_size, tx.shape[0]),
                                        shuffle=False, augment=False, seed=cfg.seed,
                                        device=self.device, channels_last=self.channels_last,
                                        drop_last=False)

        # model / flat buffers / optimizer ------------------------------------------------------
        model = build_model(net, info["classes"]).to(self.device)
        if self.channels_last:
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        # pointer-mode gradients (read in place by the HIP kernels) for the all-to-all exchange
        # and local SGD (its local steps read them through the same pointer tables); the
        # parameter server keeps flat gradient views
        ptr_grads = (self.cuda and cfg.topology == "allgather"
                     and os.environ.get("EWDML_GRAD_VIEWS") != "1")
        bf16_params = (ptr_grads and cfg.amp == "bf16" and cfg.param_dtype == "auto"
                       and not self.amp_kept_fp32)
        # weight gradients beside the backward-data chain (ops/conv.py), switched on around this
        # trainer's backward passes only: deep conv nets
        n_conv = sum(isinstance(m, torch.nn.Conv2d) for m in model.modules())
        self.wgrad_stream = bool(self.cuda and cfg.fused_nn == "on" and (
            cfg.wgrad_stream == "on"
            or (cfg.wgrad_stream == "auto" and ptr_grads and n_conv >= 30)))
        bucket_bytes = int(cfg.bucket_mb * (1 << 20))
        # --hip-graph auto for the all-to-all exchange: overlap large dense collectives with
        # backward at N > 1 (segmented graphs), one graph otherwise (plan_graph_mode); decided
        # here because the segmented step wants smaller buckets
        self.graph_plan = None
        if (cfg.hip_graph == "auto" and self.cuda and not cfg.sync_debug
                and cfg.topology == "allgather" and cfg.sync_every == 1 and not cfg.select_best):
            # EWDML_PLAN_AS_WORLD (test hook): plan as if the job had that many ranks, so the
            # N > 1 decision runs end to end on a one-GPU box (world of one, real communicator)
            plan_world = int(os.environ.get("EWDML_PLAN_AS_WORLD", self.world))
            self.graph_plan = plan_graph_mode(
                plan_world, self.comm.kind, cfg.compress,
                sum(p.numel() for p in model.parameters() if p.requires_grad),
                bits=cfg.qsgd_bits, overlap=cfg.overlap, bucket_bytes=bucket_bytes,
                model=cfg.network, topk_ratio=cfg.topk_ratio,
                dtype="fp32" if self.amp_kept_fp32 else
                {"bf16": "bf16", "fp16": "fp16"}.get(cfg.amp, "fp32"))
            bucket_bytes = self.graph_plan["bucket_bytes"]
        self.flat = FlatModel(model, bucket_bytes=bucket_bytes,
                              attach_grads=not ptr_grads, bf16_params=bf16_params)
        sync_params(self.flat, self.comm)
        sync_buffers(model, self.comm)
        lr = cfg.lr * (n_workers if cfg.lr_scale_world else 1)
        self.base_lr = lr
        self.n_workers = n_workers
        self.opt = make_optimizer(cfg.optimizer, self.flat, lr=lr, momentum=cfg.momentum,
                                  dampening=cfg.dampening, weight_decay=cfg.weight_decay,
                                  nesterov=cfg.nesterov)

        # exchange ---------------------------------------------------------------------------------
        ckw = dict(ratio=cfg.topk_ratio, levels=cfg.qsgd_levels, bits=cfg.qsgd_bits,
                   norm=cfg.qsgd_norm, seed=cfg.seed, dense_below=cfg.topk_dense_below)
        if cfg.topk_warmup and cfg.topology != "allgather":
            raise ValueError("--topk-warmup needs the all-to-all topology")
        if cfg.topology == "ps":
            self.exchange = PSExchange(self.flat, self.comm, make_codec(cfg.compress, **ckw),
                                       make_codec(cfg.pull_compress or cfg.compress, **ckw),
                                       self.opt, pull=cfg.pull,
                                       aggregate=cfg.num_aggregate if cfg.mode == "kill" else None,
                                       kill_threshold=cfg.kill_threshold if cfg.mode == "kill"
                                       else None)
        elif cfg.topology == "sharded":
            self.exchange = ShardedPSExchange(self.flat, self.comm, cfg.compress, self.opt, **ckw)
        else:
            # captured steps keep the encode + collectives on the step's own stream: a side-stream
            # fork makes the graph a DAG, which ROCm 7.2 replays node by node from the host (~7.9
            # ms per ResNet-50 step against 0.16 ms linear: profiles/ab/bucket_overlap.txt).
            # Eager steps overlap encode with backward on a side stream.
            side = (self.cuda and not cfg.phase_timing  # phase marks partition ONE stream
                    and (cfg.hip_graph == "off" or os.environ.get("EWDML_SIDE_STREAM") == "1"))
            self.exchange = GradientExchange(self.flat, self.comm,
                                             make_codec(cfg.compress, **ckw), self.opt,
                                             overlap=cfg.overlap,
                                             error_feedback=cfg.error_feedback,
                                             predivide=cfg.predivide, side_stream=side,
                                             # local SGD compresses model deltas / steps locally:
                                             # no sender-side momentum there
                                             ef_mode=cfg.ef_mode if (cfg.sync_every == 1 and
                                                                     not cfg.select_best)
                                             else "plain")
            if cfg.sync_every > 1 or cfg.select_best:
                self.exchange = LocalSGDExchange(self.exchange, cfg.sync_every, cfg.sync_mode,
                                                 cfg.select_best, score_fn=self._holdout_score)

        self.amp_dtype = {"bf16": torch.bfloat16, "fp16": torch.float16}.get(cfg.amp)
        if self.amp_kept_fp32:
            self.amp_dtype = None
            self.log.info("--amp bf16: the model's fused fp32 step is faster than its bf16 "
                          "path; training in fp32")
        self.compute_dtype = {torch.bfloat16: "bf16", torch.float16: "fp16"}.get(
            self.amp_dtype, "fp32")
        self.graph_mode = cfg.hip_graph if (self.cuda and not cfg.sync_debug) else "off"
        self.local_sgd = isinstance(self.exchange, LocalSGDExchange)
        if self.local_sgd and cfg.select_best:
            self._holdout_batch()
        # split graphs around eager collectives: the parameter server's workers (without k-of-n)
        # and the sharded exchange (graph A: forward, backward, push encodes -> eager all-to-all,
        # owner average + re-encode, all-gather -> graph B: decode + update)
        ps_split = ((isinstance(self.exchange, PSExchange) and self.exchange.k == self.world - 1)
                    or isinstance(self.exchange, ShardedPSExchange))
        self.ps_graph = ps_split
        if self.graph_mode == "auto":
            # graphs wherever the step can be captured: the all-to-all exchange, local SGD's
            # local steps (its sync steps -- compressed delta, host-side best-worker choice --
            # run eagerly), the parameter server's workers and the sharded exchange (graph A:
            # forward, backward, push encode -> eager collectives -> graph B: pull decode +
            # update); the k-of-n arrival polling stays eager
            if self.graph_plan is not None:
                self.graph_mode = self.graph_plan["mode"]
            elif isinstance(self.exchange, GradientExchange) or self.local_sgd:
                self.graph_mode = "full"
            else:
                self.graph_mode = "split" if ps_split else "off"
        if self.graph_mode != "off" and not (isinstance(self.exchange, GradientExchange) or
                                             (self.local_sgd and self.graph_mode == "full") or
                                             (ps_split and self.graph_mode == "split")):
            raise ValueError("--hip-graph: all-to-all topology (local SGD: full only; parameter "
                             "server without k-of-n and sharded: split only)")
        if (self.graph_mode in ("full", "segmented") and self._pg_collectives()
                and not self.local_sgd and not self.ps_graph):
            # the step's collectives on the process group: Gloo's CUDA collectives cannot be
            # captured, and a captured RCCL process-group collective leaves a work event recorded
            # in the capture that the group's watchdog thread then queries (hipErrorCapturedEvent
            # kills the process) -- graph the compute, issue the collectives between the graphs
            self.graph_mode = "split"
        if (cfg.phase_timing and cfg.hip_graph == "auto" and self.graph_mode == "full"
                and not self.local_sgd):
            # one graph has no inside to time: cut it at the collectives (graph A -> eager
            # collectives -> graph B) so the communication / computation split is measured
            self.graph_mode = "split"
        if (self.world == 1 and type(self.exchange) is GradientExchange
                and len(self.flat.buckets) == 1 and self.graph_mode in ("full", "off")
                and os.environ.get("EWDML_LOCAL_APPLY", "1") != "0"):
            # a world of one: the top-k write pass applies the update (the all-gather of one
            # payload is that payload: no decode launch).  One bucket, encoded once backward has
            # produced every gradient (an earlier bucket's encode would move parameters that the
            # rest of backward still reads); EWDML_LOCAL_APPLY=0: decode
            self.exchange.enable_local_apply()
        # --phase-timing: the step's phase clock, shared with the exchange (engine.Stopwatch)
        self.clock = Stopwatch(self.cuda) if cfg.phase_timing else None
        for e in (self.exchange, getattr(self.exchange, "inner", None)):
            if e is not None and hasattr(e, "clock"):
                e.clock = self.clock
        self.overlap_splits = (self.graph_plan["splits"] if (self.graph_plan is not None and
                                                             self.graph_mode == "segmented")
                               else cfg.overlap_splits)
        if self.graph_mode == "segmented":  # collectives on their own stream, beside backward
            self.exchange.comm_stream = torch.cuda.Stream(device=self.device)
        self._graphs = None
        # (U, graph, loss, out): U consecutive steps captured as one graph (train_steps)
        self._ugraph = None
        self._unroll_bad = False
        # local SGD keeps two captured steps, "local" and (model mode, own communicator) "sync";
        # the idle one waits here with its static inputs and outputs
        self._gkind, self._gslots = "local", {}
        self.captures = 0  # graph captures so far (a schedule change should not force one)
        self._in_graph_batch = False
        self._key_synced = False
        # Graph mode: warmup, capture and replay all run on ONE dedicated stream, so MIOpen /
        # hipBLASLt create their per-stream handles and workspaces during the eager warmup and not
        # inside the capture (lazy per-stream init inside a capture crashes capture_end).
        self.gstream = torch.cuda.Stream(device=self.device) if self.graph_mode != "off" else None
        # data-plane failure detection: the own RCCL communicator's collectives are bounded by
        # --comm-timeout through the native step watchdog (abort + non-zero exit)
        if self.cuda:
            self.comm.arm_watchdog(cfg.comm_timeout)
        self.step = 0
        self.epoch = 0
        self.fault = None
        if cfg.inject_fault:
            r, s = cfg.inject_fault.split(":")
            self.fault = (int(r), int(s))
        if cfg.resume:
            self._resume()

    # --------------------------------------------------------------------------------------------
    def autocast(self):
        if self.amp_dtype is None:
            return contextlib.nullcontext()
        return torch.autocast(device_type=self.device.type, dtype=self.amp_dtype,
                              enabled=self.cuda or self.amp_dtype == torch.bfloat16,
                              cache_enabled=self.graph_mode == "off")

    def _range(self, name):
        """roctx range (``--roctx``; shows up in ``rocprofv3 --marker-trace``)."""
        if not (self.cfg.roctx and self.cuda):
            return contextlib.nullcontext()
        return torch.cuda.nvtx.range(name)

    def _defer_batch(self) -> bool:
        """The fused loader's batch may be formed by the model's fused step (LeNet: its conv
        launch, ops/lenet.py) instead of its own launch (EWDML_BATCH_IN_MODEL=0: never)."""
        return (os.environ.get("EWDML_BATCH_IN_MODEL", "1") != "0"
                and getattr(self.model, "fused_loss", None) is not None and self.cuda
                and self.cfg.fused_nn == "on" and self.amp_dtype is None)

    def forward_backward(self, x, y):
        self.flat.zero_grad()
        self.exchange.begin()
        fused = None
        # a model with a fused training step of its own (LeNet: ops/lenet.py) returns the loss
        # and logits from it, or None where it does not apply
        fl = getattr(self.model, "fused_loss", None)
        if fl is not None and self.cuda and self.cfg.fused_nn == "on" and self.amp_dtype is None:
            with self._range("forward"):
                fused = fl(x, y)
        if fused is not None:
            loss, out = fused
            if self.clock is not None:
                self.clock.mark("forward")
        else:
            ldr = getattr(x, "_ew_batch", None)
            if ldr is not None:  # a deferred batch nobody formed: its kernel now
                ldr.flush()
            with self._range("forward"), self.autocast():
                out = self.model(x)
            if self.clock is not None:
                self.clock.mark("forward")
            if self.cuda and self.cfg.fused_nn == "on":
                from ..ops.nn import cross_entropy  # one HIP kernel per direction

                loss = cross_entropy(out, y)
            else:
                loss = F.cross_entropy(out.float(), y)
        with self._range("backward+encode"):
            # a persistent d(loss)/d(loss) = 1: backward() would fill a fresh one every step
            seed = getattr(self, "_loss_seed", None)
            if seed is None or seed.device != loss.device or seed.dtype != loss.dtype:
                seed = self._loss_seed = torch.ones((), dtype=loss.dtype, device=loss.device)
                if self.cuda:  # never written: the cross-entropy kernel may pre-form its grad
                    from ..ops.nn import set_unit_grad

                    set_unit_grad(seed)
            if self.cuda:
                from ..ops.conv import join_wgrad, set_wgrad_stream

                set_wgrad_stream(self.wgrad_stream)
                try:
                    loss.backward(seed)
                finally:
                    set_wgrad_stream(False)
                    join_wgrad()  # weight gradients issued on the side stream
            else:
                loss.backward(seed)
        if self.clock is not None:
            self.clock.mark("backward")
        return loss, out

    def stream_ctx(self):
        """Context of the stream the training step runs on (the graph stream in graph mode)."""
        if self.gstream is None:
            return contextlib.nullcontext()
        return torch.cuda.stream(self.gstream)

    def _drop_graphs(self):
        """Forget every captured step (the next graphed step re-captures)."""
        self._graphs = None
        self._gslots = {}
        self._ugraph = None

    def _graph_kind(self):
        """Local SGD: make the captured graph of this step's kind current."""
        kind = "sync" if self.exchange.is_sync else "local"
        if kind == self._gkind:
            return
        fields = ("_graphs", "_gloss", "_gout", "_gbytes", "_gx", "_gy", "_in_graph_batch")
        self._gslots[self._gkind] = tuple(getattr(self, f, None) for f in fields)
        vals = self._gslots.pop(kind, (None,) * len(fields))
        for f, v in zip(fields, vals):
            setattr(self, f, v)
        if self._in_graph_batch is None:
            self._in_graph_batch = False
        self._gkind = kind

    def _pg_collectives(self) -> bool:
        """The step's data-plane collectives go through the process group (Gloo, or RCCL when
        the own communicator is off): not capturable in a HIP graph."""
        return self.comm.kind == "process-group"

    def _sync_graphable(self) -> bool:
        # model mode: delta encode, all-gather and the on-device best-worker choice are all
        # device work on the own communicator; grad mode's dense re-broadcast roots at a
        # host-chosen rank
        if self._pg_collectives():
            return False
        return self.exchange.mode == "model"

    def train_step(self, x=None, y=None):
        """One synchronous step.  Returns (loss tensor, logits) (server: (None, None))."""
        if self.local_sgd and self.graph_mode != "off":
            self._graph_kind()
        if self.clock is not None:
            self.clock.reset()
            self.clock.mark("start")
        if self.gstream is None:
            out = self._train_step(x, y)
        elif self._graphs is not None and len(self._graphs) == 1 and _SAME_STREAM_REPLAY:
            # a captured full-step graph replays on the caller's stream: no per-step event hop
            # to the graph stream and back (re-captures name their capture stream themselves)
            out = self._train_step(x, y)
        else:
            gs = self.gstream  # a failed capture drops self.gstream inside the step
            gs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(gs):
                out = self._train_step(x, y)
            torch.cuda.current_stream().wait_stream(gs)
        self.comm.watch()  # the step's collectives are behind this point of the stream
        if self.clock is not None:
            self.clock.mark("other")  # anything after the last phase mark (host bookkeeping)
        return out

    def train_steps(self, n: int, unroll: int = 1):
        """``n`` synchronous steps; returns the last one's (loss, out).  With ``unroll`` U > 1 and
        a captured single-graph step (``--hip-graph full``, fused loader, constant schedules),
        runs of U steps replay one graph holding U copies of the step: the same kernels and
        collectives, one graph launch boundary (~7.7 us on MI355X,
        ``tools/probes/launch_floor.py``) per U steps instead of per step.  Steps that do not fit a
        run of U (the remainder, an epoch boundary) replay the one-step graph."""
        out = None
        while n > 0:
            if unroll > 1 and n >= unroll and self._unroll_ok(unroll) and \
                    (self._ugraph is not None and self._ugraph[0] == unroll
                     or self.prepare_unrolled(unroll)):
                out = self._unrolled_step()
                n -= unroll
            else:
                out = self.train_step()
                n -= 1
        return out

    def prepare_unrolled(self, unroll: int) -> bool:
        """Capture the U-step graph now (outside a timed region) if :meth:`train_steps` would use
        it; True when it is ready."""
        if unroll > 1 and not self._unroll_bad and self._unroll_ok(unroll, pos=False):
            if self._ugraph is None or self._ugraph[0] != unroll:
                err = None
                try:
                    self._capture_unrolled(unroll)
                except Exception as e:  # noqa: BLE001 - the one-step graph keeps running
                    err = e
                # every rank or none (the graph holds the step's collectives)
                if self.comm.all_reduce_scalars([0.0 if err is None else 1.0], op="max")[0]:
                    self._ugraph = None
                    self._unroll_bad = True
                    if err is not None:  # a failed capture can leave its stream capturing
                        self.gstream = torch.cuda.Stream(device=self.device)
                        ge = getattr(self.exchange, "inner", self.exchange)
                        if getattr(ge, "side", None) is not None:
                            ge.side = torch.cuda.Stream(device=self.device)
                    torch.cuda.synchronize()
                    self.log.info(f"unrolled graph capture failed ({err!r} on this rank); "
                                  "one graph per step")
                    return False
            return True
        return False

    def _unroll_ok(self, unroll: int, pos: bool = True) -> bool:
        cfg = self.cfg
        ok = (self.graph_mode == "full" and self._graphs is not None and len(self._graphs) == 1
              and self._in_graph_batch and self.loader is not None and self.loader.fused
              and self.clock is None and not self.local_sgd and not self.is_server
              and not self.ps_graph and self.fault is None and self.gstream is not None
              and not (cfg.lr_warmup_epochs > 0 or cfg.lr_decay_epochs)
              and not [v for v in cfg.topk_warmup.split(",") if v.strip()])
        if ok and pos:  # no epoch roll-over inside the run (the permutation is host-driven)
            self.loader.begin_step()
            ok = self.loader._pos + unroll <= self.loader.batches_per_epoch
        return ok

    def _capture_unrolled(self, unroll: int):
        ex = self.exchange
        saved = (ex.step_idx, self.opt.steps)
        mode = os.environ.get("EWDML_GRAPH_CAPTURE_MODE", "thread_local")
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        # the returned loss / logits live outside the shared pool: one-step replays interleaved
        # with this graph's may reuse the blocks of its temporaries (PyTorch guarantees pool
        # sharing only for replays in capture order), and a caller may still hold the values
        keep = tuple(None if t is None else torch.empty_like(t)
                     for t in (self._gloss, self._gout))
        try:
            # the one-step graph's pool: the two never run at once (same stream, in order)
            with torch.cuda.graph(g, pool=self._graphs[0].pool(), stream=self.gstream,
                                  capture_error_mode=mode):
                try:
                    for _ in range(unroll):
                        self._gx, self._gy = self.loader.emit(defer=self._defer_batch())
                        loss, out = self.forward_backward(self._gx, self._gy)
                        ex.finish()
                    loss, out = (t if k is None else k.copy_(t)
                                 for k, t in zip(keep, (loss, out)))
                except BaseException:
                    self._rejoin_side()
                    raise
        finally:
            ex.step_idx, self.opt.steps = saved
        self._ugraph = (unroll, g, loss, out)

    def _unrolled_step(self):
        unroll, g, loss, out = self._ugraph
        ex = self.exchange
        for _ in range(unroll):
            self.loader.advance()
        if not self._key_synced:
            ex.set_device_key()
            self._key_synced = True
        if _SAME_STREAM_REPLAY:  # as the one-step graph (train_step)
            with self._range("graph_steps"):
                g.replay()
        else:
            gs = self.gstream
            gs.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(gs):
                with self._range("graph_steps"):
                    g.replay()
            torch.cuda.current_stream().wait_stream(gs)
        self.comm.watch()
        ex.step_idx += unroll
        self.opt.steps += unroll
        ex.last = self._gbytes
        self.step += unroll
        return loss, (out, self._gy)

    def close(self):
        """Release the exchange hooks, the watchdog and the own RCCL communicator (collective:
        every rank calls it).  The process group stays up."""
        self.exchange.close()
        if self.cuda and getattr(self, "_loss_seed", None) is not None:
            from ..ops.nn import set_unit_grad

            set_unit_grad(None)
            self._loss_seed = None
        if self._own_comm:
            self.comm.close()

    def lr_at(self, step: int) -> float:
        """Learning-rate schedule: linear warmup from lr/W (or --lr-warmup-start x lr) over
        --lr-warmup-epochs (Horovod's LearningRateWarmupCallback, tensorflow_mnist.py:65-66;
        Goyal et al.'s gradual warm-up), then step decay."""
        cfg = self.cfg
        spe = len(self.loader) if self.loader is not None else 1
        epoch = step / max(1, spe)
        lr = self.base_lr
        if cfg.lr_warmup_epochs > 0 and epoch < cfg.lr_warmup_epochs:
            lo = lr * cfg.lr_warmup_start if cfg.lr_warmup_start is not None \
                else lr / max(1, self.n_workers)
            lr = lo + (lr - lo) * epoch / cfg.lr_warmup_epochs
        for e in [float(v) for v in cfg.lr_decay_epochs.split(",") if v.strip()]:
            if epoch >= e:
                lr *= cfg.lr_decay
        return lr

    def ratio_at(self, step: int):
        """Top-k density at ``step``: the --topk-warmup stages, each an equal share of
        --topk-warmup-epochs, then --topk-ratio (DGC's exponentially decreasing density)."""
        cfg = self.cfg
        stages = [float(v) for v in cfg.topk_warmup.split(",") if v.strip()]
        if not stages:
            return cfg.topk_ratio
        spe = len(self.loader) if self.loader is not None else 1
        span = cfg.topk_warmup_epochs * max(1, spe)
        i = int(step * len(stages) // max(1.0, span)) if span > 0 else len(stages)
        return stages[i] if i < len(stages) else cfg.topk_ratio

    def _apply_ratio_schedule(self):
        ex = getattr(self.exchange, "inner", self.exchange)
        if not self.cfg.topk_warmup or not hasattr(ex, "set_ratio"):
            return
        if ex.set_ratio(self.ratio_at(self.step)):
            self._drop_graphs()  # payload sizes changed: re-capture at this step (every rank)

    def _train_step(self, x=None, y=None):
        if self.fault is not None and self.fault == (self.rank, self.step):
            raise FaultInjected(f"injected fault on rank {self.rank} at step {self.step}")
        self._apply_ratio_schedule()
        if self.cfg.lr_warmup_epochs > 0 or self.cfg.lr_decay_epochs:
            lr = self.lr_at(self.step)
            if lr != self.opt.lr:
                self.opt.lr = lr  # on the GPU also into the device lr the kernels read
                if self._graphs is not None and getattr(self.opt, "lr_t", None) is None:
                    self._drop_graphs()  # the lr is a kernel argument: re-capture (all ranks)
        if self.is_server:
            if not self.model.training:
                self.model.train()
            self.exchange.finish()
            self.step += 1
            return None, None
        if not self.model.training:  # recursive; ~0.2 ms of host time per step otherwise
            self.model.train()
        graphed = self.graph_mode != "off" and self.step >= self.cfg.graph_warmup
        if graphed and self.local_sgd and self.exchange.is_sync and not self._sync_graphable():
            graphed = False  # dense re-sync / best-worker choice (host decisions): eager
        if x is None and graphed and self.loader.fused:
            # the batch kernel is part of the graph: only the host-side epoch bookkeeping here
            if self._graphs is not None and not self._in_graph_batch:
                self._drop_graphs()  # captured around an explicit batch: re-capture
            self.loader.begin_step()
            if self._graphs is None and not self._try_capture(None, None):
                return self._train_step()  # capture failed on some rank: all run eager
            return self._graph_step(None, None)
        if x is None:
            x, y = self.loader.next(static=True)
        if graphed:
            if self._graphs is None and not self._try_capture(x, y):
                return self._train_step(x, y)  # capture failed on some rank: all run eager
            return self._graph_step(x, y)
        loss, out = self.forward_backward(x, y)
        with self._range("exchange+update"):
            self.exchange.finish()
        self.step += 1
        return loss, (out, y)

    # -- HIP graph execution ----------------------------------------------------------------------
    def _try_capture(self, x, y) -> bool:
        """Capture on every rank, then agree (eager all-reduce) whether all succeeded; otherwise
        every rank drops its graphs and continues eagerly, so no rank replays collectives that a
        peer would not match."""
        err = None
        try:
            self._capture(x, y)
        except Exception as e:  # noqa: BLE001 - any capture failure falls back to eager
            err = e
        if self.ps_graph:
            # a parameter-server worker's graphs hold no collectives (the gather / broadcast run
            # eagerly between them), so one worker falling back to eager cannot desynchronise
            # the protocol -- and the server, which captures nothing, is not there to agree
            bad = err is not None
        else:
            bad = self.comm.all_reduce_scalars([0.0 if err is None else 1.0], op="max")[0]
        if bad:
            ex = self.exchange
            self._drop_graphs()
            self.graph_mode = "off"
            for e in (ex, getattr(ex, "inner", None)):
                if e is not None:
                    e.use_dev_key = e.defer_comm = e._active = e.dev_key_advance = False
            # a stream forked into an aborted capture (the encode side stream, a backend's
            # internal stream) can stay in capture mode: continue on fresh streams
            self.gstream = None
            ge = getattr(ex, "inner", ex)  # the exchange that owns the encode side stream
            if getattr(ge, "side", None) is not None:
                ge.side = torch.cuda.Stream(device=self.device)
            try:
                torch.cuda.synchronize()
            except Exception as e:  # noqa: BLE001 - the eager step below reports a real fault
                self.log.info(f"synchronize after the failed capture: {e!r}")
            self.log.info(f"HIP graph capture failed ({err!r} on this rank); running eagerly")
            return False
        return True

    def _capture(self, x, y):
        """Capture the whole training step into HIP graph(s) (static input buffers; the batch
        position and the QSGD RNG key advance in device memory from one replay to the next).

        ``full``: one graph = zero grads, fwd, bwd, hook-driven encode on the side stream, RCCL
        collectives, fused decode+SGD.  ``split``: graph A (through encode) -> eager RCCL calls ->
        graph B (decode+SGD), for process groups whose collectives cannot be captured.
        ``segmented``: linear compute segments split at bucket boundaries, one encode + collective
        graph per bucket on the comm stream, and the apply graph (``SegmentedCapture``): the
        collectives overlap the rest of backward."""
        ex = self.exchange
        self.captures += 1
        self._in_graph_batch = x is None  # fused loader: the batch kernel is captured too
        if x is not None:
            self._gx = x.clone()
            self._gy = y.clone()
        ex.use_dev_key = True
        ex.dev_key_advance = True  # the captured decode advances the device RNG key per replay
        self._key_synced = False
        inner = getattr(ex, "inner", None)  # local SGD's wrapped exchange
        saved = (ex.step_idx, self.opt.steps, inner.step_idx if inner is not None else 0)
        if inner is not None:
            # the sync graph's delta encode reads its RNG key from device memory, set before
            # every replay (_graph_step)
            inner.use_dev_key = self._gkind == "sync"
        # thread_local: only this thread's capture-unsafe HIP calls are refused.  In "global" mode
        # the RCCL process group's watchdog thread, which polls its work events, hits
        # hipErrorStreamCaptureUnsupported whenever a poll lands inside our capture, and that
        # error terminates the process (seen with a real RCCL communicator).
        mode = os.environ.get("EWDML_GRAPH_CAPTURE_MODE", "thread_local")
        torch.cuda.synchronize()
        try:  # the counters come back on the failure path too (eager fallback stays in step)
            if self.graph_mode == "full":
                # EWDML_GRAPH_DUMP=<path>: the captured step's shape (node / edge counts, forks,
                # joins, node types) as JSON at <path> and the DOT file at <path>.dot
                dump = os.environ.get("EWDML_GRAPH_DUMP")
                g = torch.cuda.CUDAGraph(keep_graph=True) if dump else torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=self.gstream, capture_error_mode=mode):
                    try:
                        if self._in_graph_batch:
                            self._gx, self._gy = self.loader.emit(defer=self._defer_batch())
                        loss, out = self.forward_backward(self._gx, self._gy)
                        ex.finish()
                    except BaseException:
                        self._rejoin_side()
                        raise
                if dump:
                    import json

                    from .. import ops

                    info = ops.graph_info(g.raw_cuda_graph(), dump + ".dot")
                    info["comm"] = self.comm.kind
                    with open(dump, "w") as f:
                        json.dump(info, f)
                    g.instantiate()
                self._graphs = (g,)
            elif self.graph_mode == "segmented":
                # device hand-offs unless --phase-timing marks the phases between the graphs
                # (EWDML_SEG_HANDOFF=event: cross-stream events and an apply graph)
                dev = (self.clock is None
                       and os.environ.get("EWDML_SEG_HANDOFF", "device") != "event")
                seg = SegmentedCapture(self.gstream, ex.comm_stream, mode="relaxed",
                                       total_bytes=4 * self.flat.numel,
                                       splits=self.overlap_splits, device_handoff=dev)
                ex.seg = seg
                try:
                    seg.begin()
                    if self._in_graph_batch:
                        self._gx, self._gy = self.loader.emit(defer=self._defer_batch())
                    loss, out = self.forward_backward(self._gx, self._gy)
                    ex.launch_pending()
                    if dev:  # the apply in the last segment, behind the comm graphs
                        ex.seg = None
                        seg.join_comms()
                        ex._active = False
                        with torch.cuda.stream(self.gstream):
                            ex.apply()
                    seg.end()
                except BaseException:
                    seg.abort()
                    raise
                finally:
                    ex.seg = None
                ex._active = False
                if not dev:
                    # the apply waits for every comm graph (replay joins the comm stream first)
                    ga = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(ga, pool=seg.pool, stream=self.gstream,
                                          capture_error_mode=mode):
                        ex.apply()
                    seg.apply = ga
                self._graphs = ("segmented", seg)
            else:
                ex.defer_comm = True
                ga = torch.cuda.CUDAGraph()
                with torch.cuda.graph(ga, stream=self.gstream, capture_error_mode=mode):
                    try:
                        if self._in_graph_batch:
                            self._gx, self._gy = self.loader.emit(defer=self._defer_batch())
                        loss, out = self.forward_backward(self._gx, self._gy)
                        ex.launch_pending()
                    except BaseException:
                        self._rejoin_side()
                        raise
                    ex.join_side()
                ex._active = False
                gb = torch.cuda.CUDAGraph()
                with torch.cuda.graph(gb, pool=ga.pool(), stream=self.gstream,
                                      capture_error_mode=mode):
                    ex.apply()
                self._graphs = (ga, gb)
        finally:
            ex.step_idx, self.opt.steps = saved[:2]
            if inner is not None:
                inner.step_idx = saved[2]
        self._gloss, self._gout = loss, out
        self._gbytes = ex.bytes_per_step()

    def _rejoin_side(self):
        """Join the encode side stream back into a capture being aborted: hipStreamEndCapture
        refuses to close a capture with an unjoined fork and leaves the stream capturing."""
        side = getattr(getattr(self.exchange, "inner", self.exchange), "side", None)
        if side is None:
            return
        with torch.cuda.stream(side):
            forked = torch.cuda.is_current_stream_capturing()
        if forked:
            torch.cuda.current_stream().wait_stream(side)

    def _graph_step(self, x, y):
        ex = self.exchange
        if self._in_graph_batch:
            if x is not None:  # an explicit batch after an in-graph-batch capture: re-capture
                self._drop_graphs()
                return self._train_step(x, y)
            self.loader.advance()
        elif x is not self._gx:
            self._gx.copy_(x)
            self._gy.copy_(y)
        if self.ps_graph:
            ex.set_device_key()  # the push encode's key of this step (no decode advances it)
        elif not self._key_synced and not self.local_sgd:
            ex.set_device_key()  # once per capture; the replays advance the key on the device
            self._key_synced = True
        elif self.local_sgd and self._gkind == "sync":
            # the delta encode's key of this sync (the eager path's inner.finish count)
            ex.inner.set_device_key(ex.inner.step_idx)
            ex.inner.step_idx += 1
        clk = self.clock
        if len(self._graphs) == 1:
            with self._range("graph_step"):
                self._graphs[0].replay()
            if clk is not None:
                clk.mark("step")  # one graph: no phases inside
        elif self._graphs[0] == "segmented":
            with self._range("graph_step"):
                self._graphs[1].replay(clk)
        else:
            self._graphs[0].replay()
            if clk is not None:
                clk.mark("compute")  # graph A: forward, backward, encode
            ex.communicate()
            ex.wait()
            if clk is not None:
                clk.mark("collective")
            self._graphs[1].replay()
            if clk is not None:
                clk.mark("decode_update")  # graph B
        ex.step_idx += 1
        self.opt.steps += 1
        # a local step sends nothing
        ex.last = StepStats() if (self.local_sgd and self._gkind == "local") else self._gbytes
        self.step += 1
        return self._gloss, (self._gout, self._gy)

    @torch.no_grad()
    def evaluate(self, max_batches=None):
        """Test loss / top-1 / top-5 of this rank's replica (the reference evaluator's output,
        with a correct cross-entropy instead of NLL on raw logits)."""
        self.model.eval()
        n = 0
        loss = torch.zeros((), device=self.device, dtype=torch.float64)
        c1 = torch.zeros((), device=self.device, dtype=torch.float64)
        c5 = torch.zeros((), device=self.device, dtype=torch.float64)
        self.test_loader.set_epoch(0)
        for i, (x, y) in enumerate(self.test_loader):
            if max_batches is not None and i >= max_batches:
                break
            with self.autocast():
                out = self.model(x)
            out = out.float()
            loss += F.cross_entropy(out, y, reduction="sum")
            a1, a5 = accuracy(out, y, (1, 5))
            c1 += a1 * y.shape[0] / 100.0
            c5 += a5 * y.shape[0] / 100.0
            n += y.shape[0]
        if not self.model.training:  # recursive; ~0.2 ms of host time per step otherwise
            self.model.train()
        n = max(n, 1)
        return {"test_loss": float(loss) / n, "top1": 100.0 * float(c1) / n,
                "top5": 100.0 * float(c5) / n, "samples": n}

    def _holdout_batch(self):
        """The first held-out batch as static tensors (made once, outside any capture)."""
        hb = getattr(self, "_hold_batch", None)
        if hb is None:
            self.test_loader.set_epoch(0)
            x, y = next(iter(self.test_loader))
            hb = self._hold_batch = (x.clone(), y.clone())
        return hb

    def _holdout_score(self):
        """Top-1 (%) of this replica on the first held-out batch, as a 0-dim device tensor (no
        host synchronisation: Method 6's best-worker choice runs inside the sync step's graph;
        the same batch and the same value as ``evaluate(max_batches=1)["top1"]``)."""
        x, y = self._holdout_batch()
        self.model.eval()
        with torch.no_grad(), self.autocast():
            out = self.model(x)
        self.model.train()
        return (out.float().argmax(1) == y).sum(dtype=torch.float32) * (100.0 / y.shape[0])

    # --------------------------------------------------------------------------------------------
    def state_extra(self):
        ex = self.exchange
        inner = getattr(ex, "inner", ex)
        extra = {"config": {k: v for k, v in vars(self.cfg).items()
                            if isinstance(v, (int, float, str, bool)) or v is None},
                 "world": self.world}
        for name, attr in (("ef_residual", "resid"), ("ef_velocity", "vel"),
                           ("ef_global", "gest")):
            r = getattr(inner, attr, None)
            if r is not None:
                # error-feedback residual / DGC velocity are per-rank state: keep every rank's row
                allr = torch.zeros((self.world, r.numel()), dtype=r.dtype, device=r.device)
                self.comm.all_gather(allr.view(-1), r)
                extra[name] = allr
        if self.local_sgd:
            # between syncs every replica (and its momentum) has drifted on its own: keep every
            # rank's row, the common anchor of the model-delta exchange and the sync count (the
            # delta encode's RNG stream)
            rows = {"local_params": self.flat.data}
            if getattr(self.opt, "mom", None) is not None:
                rows["local_mom"] = self.opt.mom
            for name, r in rows.items():
                allr = torch.zeros((self.world, r.numel()), dtype=r.dtype, device=r.device)
                self.comm.all_gather(allr.view(-1), r)
                extra[name] = allr
            if ex.anchor is not None:
                extra["local_anchor"] = ex.anchor
            extra["local_syncs"] = inner.step_idx
        return extra

    @property
    def buffer_src(self) -> int:
        """Rank whose BN running statistics are the model's: in the parameter-server topology
        rank 0 is the server and never runs a forward pass, so its buffers stay at their
        initial values -- the first worker's are used (the reference's workers write
        model_step_, ``distributed_worker.py:_save_model``)."""
        return 1 if (self.cfg.topology == "ps" and self.world > 1) else 0

    def save_checkpoint(self):
        """Collective (every rank calls it); rank 0 writes."""
        if self.buffer_src != 0:  # rank 0 (the server) saves the first worker's BN statistics
            sync_buffers(self.model, self.comm, src=self.buffer_src, only_to=0)
        extra = self.state_extra()
        if self.rank != 0:
            return None
        return ckpt.save(self.cfg.ckpt_dir, self.step, self.model, self.opt, self.epoch,
                         extra=extra, model_state=self.flat.master_state_dict(self.model),
                         legacy_dir=self.cfg.train_dir if self.cfg.legacy_ckpt else None)

    def _resume(self):
        path = ckpt.latest(self.cfg.ckpt_dir)
        path = self.comm.broadcast_object(path, src=0)
        if not path:
            self.log.info("resume: no checkpoint found, starting fresh")
            return
        st = ckpt.load(path)
        self.flat.load_state_dict(self.model, st["model"])
        # the params are views of the flat buffer; load_state_dict copies in place
        self.opt.load_state_dict({k: (v.to(self.device) if torch.is_tensor(v) else v)
                                  for k, v in st["optimizer"].items()})
        self.step = int(st["step"])
        self.epoch = int(st["epoch"])
        inner = getattr(self.exchange, "inner", self.exchange)
        for name, attr in (("ef_residual", "resid"), ("ef_velocity", "vel"),
                           ("ef_global", "gest")):
            r = st["extra"].get(name)
            mine = getattr(inner, attr, None)
            if r is not None and mine is not None:
                if r.dim() == 2 and r.shape[0] == self.world:
                    mine.copy_(r[self.rank].to(self.device))
                else:
                    self.log.info(f"resume: world size changed, {name} reset")
        if self.local_sgd:
            ex, ext = self.exchange, st["extra"]
            rows = [(ext.get("local_params"), self.flat.data),
                    (ext.get("local_mom"), getattr(self.opt, "mom", None))]
            for r, mine in rows:
                if r is not None and mine is not None and r.dim() == 2 and r.shape[0] == self.world:
                    mine.copy_(r[self.rank].to(self.device))
            self.flat.sync_shadow()
            if ex.anchor is not None and ext.get("local_anchor") is not None:
                ex.anchor.copy_(ext["local_anchor"].to(self.device))
            if "local_syncs" in ext:
                inner.step_idx = int(ext["local_syncs"])
        if hasattr(self.exchange, "step_idx"):
            self.exchange.step_idx = self.step
        if self.loader is not None:
            self.loader.set_epoch(self.epoch)
            self.loader.seek(self.step % len(self.loader))
        self.log.info(f"resumed from {path} at step {self.step}")

    # --------------------------------------------------------------------------------------------
    def fit(self):
        cfg = self.cfg
        total = cfg.max_steps  # the ps server has no loader: the min over ranks decides
        if self.loader is not None:
            total = min(cfg.max_steps, cfg.epochs * len(self.loader))
        total = int(self.comm.all_reduce_scalars([total], op="min")[0])
        sw = Stopwatch(self.cuda)
        t_start = time.time()
        summary = None
        prof = None
        # run totals: cumulative bytes (the reference's per-worker "total send / recieve memory",
        # src/distributed_worker.py:228-231), phase times (--phase-timing), sampled step times
        acc = {"bytes_sent": 0, "bytes_recv": 0, "payload_bytes": 0, "steps": 0,
               "phase_ms": {}, "phase_steps": 0, "step_ms": []}
        if cfg.profile and self.rank == 0:
            prof = torch.profiler.profile(
                activities=[torch.profiler.ProfilerActivity.CPU] +
                ([torch.profiler.ProfilerActivity.CUDA] if self.cuda else []))
            prof.__enter__()
        while self.step < total:
            if self.loader is not None:
                self.epoch = self.loader.epoch
            sw.reset()
            sw.mark("start")
            loss, outy = self.train_step()
            sw.mark("step")
            st = self.exchange.last
            acc["bytes_sent"] += st.wire_bytes_sent
            acc["bytes_recv"] += st.wire_bytes_recv
            acc["payload_bytes"] += st.payload_bytes
            acc["steps"] += 1
            phases = None
            if self.clock is not None:
                phases = self.clock.phases()
                for k, v in phases.items():
                    acc["phase_ms"][k] = acc["phase_ms"].get(k, 0.0) + v
                acc["phase_steps"] += 1
            if prof is not None and self.step == cfg.profile:
                prof.__exit__(None, None, None)
                prof.export_chrome_trace(os.path.join(cfg.train_dir, "trace.json"))
                prof = None
            if self.step % cfg.log_interval == 0 or self.step == total:
                rec = {"step": self.step, "epoch": self.epoch, "rank": self.rank,
                       "time_s": time.time() - t_start, "lr": self.opt.lr}
                if loss is not None:
                    out, y = outy
                    a1, a5 = accuracy(out.float(), y, (1, 5))
                    rec.update(loss=float(loss.detach()), acc1=float(a1), acc5=float(a5))
                rec["step_ms"] = sw.phases().get("step")
                acc["step_ms"].append(rec["step_ms"] or 0.0)
                if self.world > 1:  # straggler report: slowest / fastest rank's step time
                    mx, mn = self.comm.all_reduce_scalars([rec["step_ms"] or 0.0], op="max")[0], \
                        -self.comm.all_reduce_scalars([-(rec["step_ms"] or 0.0)], op="max")[0]
                    rec["step_ms_max"], rec["step_ms_min"] = mx, mn
                rec.update(byte_summary(self.exchange.last, self.world))
                # the codec's health at every log record (synchronises: the record already did):
                # a look-back failure of the top-k encode raises here
                ge = getattr(self.exchange, "inner", self.exchange)
                if hasattr(ge, "codec_health"):
                    rec.update(ge.codec_health())
                rec["bytes_sent_total"] = acc["bytes_sent"]
                rec["bytes_recv_total"] = acc["bytes_recv"]
                rec["payload_bytes_total"] = acc["payload_bytes"]
                if phases is not None:
                    rec["phase_ms"] = {k: round(v, 4) for k, v in phases.items()}
                    comm_ms, comp_ms = Stopwatch.split(phases)
                    rec["comm_ms"], rec["compute_ms"] = round(comm_ms, 4), round(comp_ms, 4)
                rec["images_per_sec_rank"] = (cfg.batch_size * 1e3 / rec["step_ms"]
                                              if rec["step_ms"] else None)
                self.log.record(rec)
                if loss is not None:
                    ph = (f" comm {rec['comm_ms']:.2f} ms compute {rec['compute_ms']:.2f} ms"
                          if phases is not None else "")
                    self.log.info(
                        f"Worker {self.rank} Step {self.step}/{total} loss {rec['loss']:.4f} "
                        f"acc@1 {rec['acc1']:.1f} acc@5 {rec['acc5']:.1f} "
                        f"payload {rec['payload_bytes_per_rank'] / 1024:.1f} KiB "
                        f"(x{(rec['compression_ratio'] or 0):.0f}) step {rec['step_ms'] or 0:.2f} ms"
                        f"{ph} sent {acc['bytes_sent'] / 2**20:.1f} MiB "
                        f"recv {acc['bytes_recv'] / 2**20:.1f} MiB")
                summary = rec
            if cfg.eval_freq and self.step % cfg.eval_freq == 0:
                if cfg.sync_bn:
                    sync_buffers(self.model, self.comm, src=self.buffer_src)
                self.save_checkpoint()
                if cfg.eval_on_ckpt and self.rank == (1 if cfg.topology == "ps" else 0):
                    ev = self.evaluate()
                    self.log.info(f"Test step {self.step}: loss {ev['test_loss']:.4f} "
                                  f"top1 {ev['top1']:.2f}% top5 {ev['top5']:.2f}%")
                    self.log.record({"step": self.step, "eval": ev})
        self.comm.barrier()
        wall = time.time() - t_start
        self.log.info(f"total time {wall:.1f}s for {total} steps")
        run_summary = self.write_summary(acc, wall)
        self.close()
        self.log.close()
        return {"steps": total, "wall_s": wall, "last": summary, "summary": run_summary}

    def write_summary(self, acc: dict, wall: float) -> dict:
        """Collective: every rank's run totals; rank 0 writes ``summary.json`` with
        each rank's figures and their mean and max over ranks -- the per-method comm / compute
        minutes the report charts (``Report.zip: VGG11 Communication and Computation Time``)."""
        n = max(1, acc["phase_steps"])
        mine = {"rank": self.rank, "steps": acc["steps"], "wall_s": wall,
                "bytes_sent_total": acc["bytes_sent"], "bytes_recv_total": acc["bytes_recv"],
                "payload_bytes_total": acc["payload_bytes"],
                "step_ms_mean": (sum(acc["step_ms"]) / len(acc["step_ms"])
                                 if acc["step_ms"] else None)}
        if acc["phase_steps"]:
            ph = {k: v / n for k, v in acc["phase_ms"].items()}
            mine["phase_ms_mean"] = ph
            comm_ms, comp_ms = Stopwatch.split(ph)
            mine["comm_ms_mean"], mine["compute_ms_mean"] = comm_ms, comp_ms
            mine["comm_s_total"] = comm_ms * acc["steps"] / 1e3
            mine["compute_s_total"] = comp_ms * acc["steps"] / 1e3
        ranks = self.comm.all_gather_object(mine)
        if self.rank != 0:
            return None

        def agg(fn):
            out = {}
            for k in ("wall_s", "bytes_sent_total", "bytes_recv_total", "payload_bytes_total",
                      "step_ms_mean", "comm_ms_mean", "compute_ms_mean", "comm_s_total",
                      "compute_s_total"):
                vals = [r[k] for r in ranks if r.get(k) is not None]
                if vals:
                    out[k] = fn(vals)
            keys = sorted({k for r in ranks for k in r.get("phase_ms_mean", {})})
            if keys:
                out["phase_ms_mean"] = {k: fn([r["phase_ms_mean"].get(k, 0.0) for r in ranks
                                               if "phase_ms_mean" in r]) for k in keys}
            return out

        cfg = self.cfg
        summary = {"world": self.world, "network": cfg.network, "dataset": cfg.dataset,
                   "method": cfg.method, "compress": cfg.compress, "topology": cfg.topology,
                   "hip_graph": self.graph_mode, "batch_size": cfg.batch_size,
                   "phase_timing": cfg.phase_timing, "ranks": ranks,
                   "mean": agg(lambda v: sum(v) / len(v)), "max": agg(max)}
        path = cfg.summary_file or os.path.join(cfg.train_dir, "summary.json")
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        import json

        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            json.dump(summary, f, indent=1)
        os.replace(tmp, path)  # atomic: a reader never sees a half-written summary
        return summary


def run(cfg: Config):
    tr = Trainer(cfg)
    return tr.fit()
