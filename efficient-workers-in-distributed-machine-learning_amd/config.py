"""Run configuration and the ``distributed_nn.py`` command line.

Every flag of the reference CLI (``src/distributed_nn.py:24-72``) is accepted with the same name
and default; the ones the reference parses but never uses keep their meaning documented below.
New flags select the exchange method, codec, topology and the MI355X execution options.

Method presets (``--method``; ``Report.zip:main.tex:80-119``):
  1  vanilla PS: push dense grads to rank 0, server steps, pull dense *weights*
  2  QSGD push, dense weight pull
  3  push + pull dense gradients (the reference's live HEAD path) -> dense all-reduce
  4  QSGD both ways
  5  top-k -> QSGD both ways (ratio --topk-ratio; the report used 0.4)
  6  method 5 + communicate every --sync-every (default 20) steps + best-worker selection
Methods 1 and 2 imply ``--topology ps``; 3-6 default to the all-to-all topology (every GPU is a
worker, no idle server); ``--topology ps`` reproduces the reference's star for any method.
"""
import argparse
import dataclasses
from dataclasses import dataclass, field
from typing import Optional


def _str2bool(v) -> bool:
    if isinstance(v, bool):
        return v
    # reference `--enable-gpu` is `type=bool`: any non-empty string is True (distributed_nn.py:68)
    return str(v).strip().lower() not in ("", "0", "false", "no", "off", "none")


# density stages of the error-feedback warm-up (DGC's exponentially decreasing density)
EF_WARMUP_STAGES = (0.25, 0.125, 0.0625, 0.03125, 0.015625)


@dataclass
class Config:
    # ---- reference flags (distributed_nn.py:24-72) -----------------------------------------
    batch_size: int = 128
    test_batch_size: int = 500
    epochs: int = 100
    max_steps: int = 10000
    lr: float = 0.01
    momentum: float = 0.5
    no_cuda: bool = False
    seed: int = 1
    log_interval: int = 10
    network: str = "LeNet"
    mode: str = "normal"  # straggler mode; 'kill' enables the --kill-threshold step timeout
    kill_threshold: float = 7.0  # seconds a PS k-of-n push may lag the k-th arrival in kill mode
    dataset: str = "MNIST"
    comm_type: str = "Bcast"  # accepted; the all-to-all exchange needs no choice here
    num_aggregate: int = 5  # PS k-of-n: with --topology ps --mode kill the server averages the
    #                         first k worker gradients to arrive (parallel/ps.py)
    eval_freq: int = 50  # checkpoint (and evaluation) cadence in steps
    train_dir: str = "output/models/"
    compress_grad: str = "compress"  # 'none' forces --compress none (reference switch)
    gather_type: str = "gather"  # accepted for compatibility
    enable_gpu: bool = False
    local_rank: Optional[int] = None
    # ---- exchange / compression ---------------------------------------------------------------
    method: Optional[int] = None
    compress: str = "topk_qsgd"  # none | fp16 | bf16 | qsgd | topk | topk_qsgd
    topk_ratio: float = 0.01
    topk_dense_below: int = 0  # tensors of <= N elements go whole (k = numel) through top-k codecs
    qsgd_levels: int = 127
    qsgd_bits: int = 8
    qsgd_norm: str = "max"  # max | l2 (the reference's L2 norm)
    topology: str = "allgather"  # allgather (all-to-all) | ps (rank-0 parameter server) |
    #                               sharded (every rank owns 1/N of each bucket: parallel/sharded.py)
    pull: str = "grad"  # ps topology: pull averaged 'grad' or server 'weights'
    pull_compress: Optional[str] = None  # ps topology: codec of the pull (default = push codec)
    sync_every: int = 1  # local SGD: exchange every H steps (method 6)
    sync_mode: str = "grad"  # grad: compressed gradient on sync steps | model: compressed delta
    sync_mode_default: bool = True  # --sync-mode not given (--method 6 then selects 'model')
    select_best: bool = False  # method 6: adopt the weights of the best-accuracy rank at sync
    # None (auto): on for the top-k codecs -- top-k at 1 % without error feedback trains 10-80x
    # slower than dense (profiles/validation/ef_stability_r03.md) -- off otherwise;
    # --no-error-feedback gives the reference's Methods 5/6 as published (no residual)
    error_feedback: Optional[bool] = None
    # dgc: momentum correction + momentum factor masking (the sender runs the momentum before
    # top-k; oracle.dgc_accumulate) | plain: residual of the raw gradient, momentum after decode
    ef_mode: str = "dgc"
    # top-k density warm-up (DGC's "exponentially decreasing sparsity"): comma-separated ratios
    # used in turn over the first --topk-warmup-epochs epochs, then --topk-ratio (e.g. "0.25,0.0625,
    # 0.015625"); each change re-plans the payloads (and re-captures a HIP graph)
    topk_warmup: str = ""
    topk_warmup_epochs: float = 2.0
    # auto: --error-feedback with a top-k codec brings its stability recipe unless set explicitly:
    # the density warm-up 25 % -> 12.5 % -> 6.25 % -> 3.125 % -> 1.5625 % (stages above
    # --topk-ratio) over --topk-warmup-epochs, and a linear lr warm-up from 0.1 lr over 2 epochs
    # (measured on ResNet-50: profiles/validation/ef_stability_r03.md) | none
    ef_warmup: str = "auto"
    bucket_mb: float = 16.0
    overlap: bool = True
    overlap_splits: int = 1  # --hip-graph segmented: comm graphs per step (split points)
    predivide: float = 1.0  # Horovod gradient_predivide_factor
    sync_bn: bool = False  # broadcast BN running stats from rank 0 at every checkpoint/eval
    # ---- optimizer -------------------------------------------------------------------------------
    optimizer: str = "sgd"
    weight_decay: float = 0.0
    dampening: float = 0.0
    nesterov: bool = False
    lr_scale_world: bool = False  # Horovod: lr *= world size
    lr_warmup_epochs: float = 0.0  # Horovod LearningRateWarmupCallback: lr/W -> lr linearly
    lr_warmup_start: Optional[float] = None  # warm-up's first lr as a fraction of lr (None: 1/W)
    lr_decay_epochs: str = ""  # e.g. "30,60,90": multiply lr by --lr-decay at these epochs
    lr_decay: float = 0.1
    # ---- execution -------------------------------------------------------------------------------
    device: str = "auto"  # auto | cuda | cpu
    # none (fp32 compute: the reference's precision, the default) | bf16 | fp16 (autocast compute
    # dtype; master weights fp32 either way)
    amp: str = "none"
    param_dtype: str = "auto"  # auto: conv/linear weights kept in bf16 (fp32 master) under bf16
    #                            autocast on the GPU all-to-all path | fp32
    channels_last: bool = False  # alias of layout="nhwc"
    layout: str = "auto"  # auto (nhwc on the GPU when the fused NHWC kernels run) | nchw | nhwc
    fused_nn: str = "on"  # on: conv-BN-ReLU-pool groups / 2x2 pools through ops/csrc/nn.hip | off
    fused_data: str = "on"  # on: training batches built by one graph-capturable kernel (GPU) | off
    # auto (full where the step can be captured, else eager) | off | split (graphs around eager
    # RCCL calls) | full (one graph) | segmented (linear compute segments + per-bucket comm graphs
    # on their own stream: collectives overlap backward)
    hip_graph: str = "auto"
    graph_warmup: int = 3  # eager steps (>= 1) before capture: MIOpen find, handles, momentum

    data_dir: Optional[str] = None  # None -> synthetic data of the dataset's shape
    synthetic_size: int = 0
    # > 0: train on the test split minus its last N samples and evaluate on those N (for data
    # directories that hold only a test split, e.g. the reference's MNIST t10k files)
    holdout_from_test: int = 0
    augment: bool = True
    # ---- checkpoint / metrics / faults -----------------------------------------------------------
    ckpt_dir: Optional[str] = None  # defaults to train_dir
    resume: bool = False
    legacy_ckpt: bool = True  # also write <train_dir>/model_step_ (the evaluator's file)
    eval_on_ckpt: bool = False
    metrics_file: Optional[str] = None  # per-step JSONL
    profile: int = 0  # wrap N steps in torch.profiler
    roctx: bool = False  # roctx ranges per phase (rocprofv3 --marker-trace)
    # per-step phase times (forward / backward / encode / collective / decode_update, or per graph
    # segment) from HIP events on the step's stream, in the JSONL and summary.json; serialises the
    # eager step (no side stream) and makes --hip-graph auto split the graph at the collectives
    phase_timing: bool = False
    # weight gradients of the MFMA convs on a second stream, beside the backward-data chain
    # (auto = on for deep conv nets, >= 30 convolutions, with pointer-mode gradients).  Measured
    # +1.7 % on ResNet-50 CIFAR and -6 % on VGG-11, but the fork / join per conv makes the
    # captured graph a DAG whose replay costs ~5 ms of host time per ResNet-50 step (0.12 ms
    # linear): off by default (profiles/ab/README.md)
    wgrad_stream: str = "off"
    summary_file: Optional[str] = None  # rank 0's run summary (default <train_dir>/summary.json)
    inject_fault: Optional[str] = None  # "rank:step" -> that rank raises at that step (tests)
    comm_timeout: float = 600.0
    sync_debug: bool = False  # synchronise after every custom kernel (race / fault localisation)
    quiet: bool = False

    def resolved(self) -> "Config":
        c = dataclasses.replace(self)
        if c.method is not None:
            m = int(c.method)
            if m not in range(1, 7):
                raise ValueError("--method must be in 1..6")
            if m == 1:
                c.topology, c.pull, c.compress = "ps", "weights", "none"
            elif m == 2:
                c.topology, c.pull, c.compress = "ps", "weights", "qsgd"
            elif m == 3:
                c.compress = "none"
            elif m == 4:
                c.compress = "qsgd"
            elif m in (5, 6):
                c.compress = "topk_qsgd"
            if m == 6:
                if c.sync_every == 1:
                    c.sync_every = 20
                c.select_best = True
                if c.sync_mode_default:  # compressed model delta, winner's delta adopted
                    c.sync_mode = "model"
        if c.compress_grad.lower() == "none":
            c.compress = "none"
        if c.error_feedback is None:
            # only the all-gather exchange keeps a residual (parallel/engine.py
            # GradientExchange); the parameter-server / sharded exchanges have none, so their
            # top-k runs keep the reference's schedule (no EF warm-up) and record no EF
            c.error_feedback = (c.compress in ("topk", "topk_qsgd")
                                and c.topology == "allgather")
        if c.ef_mode == "ef21" and c.error_feedback and c.device != "cpu" and not c.no_cuda:
            import os

            # the EF21 encode exists only in the torch oracle (flat gradient views)
            if not (os.environ.get("EWDML_ORACLE") == "1"
                    and os.environ.get("EWDML_GRAD_VIEWS") == "1"):
                import torch

                if c.device == "cuda" or torch.cuda.is_available():
                    raise ValueError("--ef-mode ef21 has no HIP encode kernel: run it on the CPU, "
                                     "or on the GPU with EWDML_ORACLE=1 EWDML_GRAD_VIEWS=1")
        if (c.ef_warmup == "auto" and c.error_feedback and c.compress in ("topk", "topk_qsgd")
                and c.sync_every == 1 and not c.select_best):
            stages = [r for r in EF_WARMUP_STAGES if r > c.topk_ratio]
            if not c.topk_warmup:
                c.topk_warmup = ",".join(f"{r:g}" for r in stages)
            if stages and c.lr_warmup_epochs <= 0:
                c.lr_warmup_epochs = 2.0
                if c.lr_warmup_start is None:
                    c.lr_warmup_start = 0.1
        if c.topology not in ("allgather", "ps", "sharded"):
            raise ValueError("--topology must be allgather, ps or sharded")
        if c.graph_warmup < 1:
            raise ValueError("--graph-warmup must be >= 1 (one eager step initialises the stream)")
        if c.ckpt_dir is None:
            c.ckpt_dir = c.train_dir
        if c.channels_last:
            c.layout = "nhwc"
        return c


def build_parser(prog="distributed_nn.py") -> argparse.ArgumentParser:
    d = Config()
    p = argparse.ArgumentParser(prog=prog, description="MI355X gradient-compressed data-parallel "
                                "training (parameter-server / all-reduce / top-k + QSGD)")
    a = p.add_argument
    # reference flags
    a("--batch-size", type=int, default=d.batch_size)
    a("--test-batch-size", type=int, default=d.test_batch_size)
    a("--epochs", type=int, default=d.epochs)
    a("--max-steps", type=int, default=d.max_steps)
    a("--lr", type=float, default=d.lr)
    a("--momentum", type=float, default=d.momentum)
    a("--no-cuda", action="store_true", default=False)
    a("--seed", type=int, default=d.seed)
    a("--log-interval", type=int, default=d.log_interval)
    a("--network", type=str, default=d.network)
    a("--mode", type=str, default=d.mode)
    a("--kill-threshold", type=float, default=d.kill_threshold)
    a("--dataset", type=str, default=d.dataset)
    a("--comm-type", type=str, default=d.comm_type)
    a("--num-aggregate", type=int, default=d.num_aggregate)
    a("--eval-freq", type=int, default=d.eval_freq)
    a("--train-dir", type=str, default=d.train_dir)
    a("--compress-grad", type=str, default=d.compress_grad)
    a("--gather-type", type=str, default=d.gather_type)
    a("--enable-gpu", type=_str2bool, default=d.enable_gpu)
    a("--local_rank", "--local-rank", dest="local_rank", type=int, default=None)
    # exchange
    a("--method", type=int, default=None, choices=range(1, 7))
    a("--compress", type=str, default=d.compress,
      choices=["none", "fp16", "bf16", "qsgd", "topk", "topk_qsgd"])
    a("--topk-ratio", type=float, default=d.topk_ratio)
    a("--topk-dense-below", type=int, default=d.topk_dense_below)
    a("--qsgd-levels", type=int, default=d.qsgd_levels)
    a("--qsgd-bits", type=int, default=d.qsgd_bits, choices=[4, 8])
    a("--qsgd-norm", type=str, default=d.qsgd_norm, choices=["max", "l2"])
    a("--topology", type=str, default=d.topology, choices=["allgather", "ps", "sharded"])
    a("--pull", type=str, default=d.pull, choices=["grad", "weights"])
    a("--pull-compress", type=str, default=None,
      choices=["none", "fp16", "bf16", "qsgd", "topk", "topk_qsgd"])
    a("--sync-every", type=int, default=d.sync_every)
    a("--sync-mode", type=str, default=None, choices=["grad", "model"])
    a("--select-best", action="store_true", default=False)
    a("--error-feedback", dest="error_feedback", action="store_true", default=None)
    a("--no-error-feedback", dest="error_feedback", action="store_false")
    a("--ef-mode", type=str, default=d.ef_mode, choices=["dgc", "plain", "local", "ef21"])
    a("--topk-warmup", type=str, default=d.topk_warmup)
    a("--topk-warmup-epochs", type=float, default=d.topk_warmup_epochs)
    a("--ef-warmup", type=str, default=d.ef_warmup, choices=["auto", "none"])
    a("--bucket-mb", type=float, default=d.bucket_mb)
    a("--no-overlap", dest="overlap", action="store_false", default=True)
    a("--overlap-splits", type=int, default=d.overlap_splits)
    a("--predivide", type=float, default=d.predivide)
    a("--sync-bn", "--sync-bn-buffers", dest="sync_bn", action="store_true", default=False)
    # optimizer
    a("--optimizer", type=str, default=d.optimizer, choices=["sgd", "adam", "amsgrad"])
    a("--weight-decay", type=float, default=d.weight_decay)
    a("--dampening", type=float, default=d.dampening)
    a("--nesterov", action="store_true", default=False)
    a("--lr-scale-world", action="store_true", default=False)
    a("--lr-warmup-epochs", type=float, default=d.lr_warmup_epochs)
    a("--lr-warmup-start", type=float, default=None)
    a("--lr-decay-epochs", type=str, default=d.lr_decay_epochs)
    a("--lr-decay", type=float, default=d.lr_decay)
    # execution
    a("--device", type=str, default=d.device, choices=["auto", "cuda", "cpu"])
    a("--amp", type=str, default=d.amp, choices=["bf16", "fp16", "none"])
    a("--param-dtype", type=str, default=d.param_dtype, choices=["auto", "fp32"])
    a("--channels-last", action="store_true", default=False)
    a("--layout", type=str, default=d.layout, choices=["auto", "nchw", "nhwc"])
    a("--fused-nn", type=str, default=d.fused_nn, choices=["on", "off"])
    a("--fused-data", type=str, default=d.fused_data, choices=["on", "off"])
    a("--hip-graph", type=str, default=d.hip_graph,
      choices=["auto", "off", "split", "full", "segmented"])
    a("--graph-warmup", type=int, default=d.graph_warmup)
    a("--data-dir", type=str, default=None)
    a("--holdout-from-test", type=int, default=d.holdout_from_test)
    a("--synthetic-size", type=int, default=0)
    a("--no-augment", dest="augment", action="store_false", default=True)
    # checkpoint / metrics / faults
    a("--ckpt-dir", type=str, default=None)
    a("--resume", action="store_true", default=False)
    a("--no-legacy-ckpt", dest="legacy_ckpt", action="store_false", default=True)
    a("--eval-on-ckpt", action="store_true", default=False)
    a("--metrics-file", type=str, default=None)
    a("--profile", type=int, default=0)
    a("--roctx", action="store_true", default=False)
    a("--phase-timing", action="store_true", default=False)
    a("--wgrad-stream", choices=["auto", "on", "off"], default=d.wgrad_stream)
    a("--summary-file", type=str, default=None)
    a("--inject-fault", type=str, default=None)
    a("--comm-timeout", type=float, default=d.comm_timeout)
    a("--sync-debug", action="store_true", default=False)
    a("--quiet", action="store_true", default=False)
    return p


def parse_args(argv=None, prog="distributed_nn.py") -> Config:
    ns = build_parser(prog).parse_args(argv)
    ns.sync_mode_default = ns.sync_mode is None
    if ns.sync_mode is None:
        ns.sync_mode = Config.sync_mode
    fields = {f.name for f in dataclasses.fields(Config)}
    return Config(**{k: v for k, v in vars(ns).items() if k in fields}).resolved()
