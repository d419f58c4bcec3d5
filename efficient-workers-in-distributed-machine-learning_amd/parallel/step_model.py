"""A step-time model for N > 1 ranks on one 8 x MI355X node, from N = 1 measurements.

The all-gather / all-reduce exchange cannot be run at N > 1 on the one-GPU development pool, so
the first scaling run needs a prediction to be checked against, and ``--hip-graph auto`` needs a
reason other than the codec's kind to choose between one graph per step (``full``: backward,
then encode, collective, decode) and per-bucket collectives overlapped with backward on a comm
stream (``segmented``).  The model:

* **Compute** -- the measured N = 1 step of the configuration (``StepProfile.full_ms``, where the
  collective is empty), plus what the N > 1 code path costs over it at world 1 (``n1_offset_ms``:
  a one-bucket top-k step applies its update in the encode at N = 1), with its decode of one
  payload replaced by the decode of N (measured at 1 / 2 / 4 / 8 payloads on one GPU:
  ``tools/probes/decode_probe.py``).  All of these are regenerated each round from that round's
  runs (``tools/step_model_calibrate.py`` -> ``parallel/n1_profiles.json``).
* **Collectives** over xGMI -- a latency term per collective plus a ring-step term per peer, and a
  bandwidth term over ``min(N - 1, 7)`` links (a fully connected 8-GPU mesh: one xGMI link to each
  peer, ~153 GB/s each) at an efficiency factor.  All-gather of P bytes per rank moves (N - 1) P
  into each rank; a ring all-reduce of S bytes moves 2 (N - 1) / N S.
* **Segmented** -- the measured N = 1 cost of segmenting the step (graph boundaries, the encode
  moved to the comm stream beside the backward GEMMs: ``seg_penalty_ms``) plus the part of the
  collectives backward cannot hide: the last split's share (it starts after backward ends) and
  whatever exceeds the backward time left after the first bucket.

Constants marked *assumed* come from the hardware sheet and typical RCCL behaviour, not from a
measurement on this node (there was none at N > 1): ``profiles/model/step_model.md`` lists them
and every N = 1 number with its source, and the first SCALE run replaces them.

The reference has no counterpart (its PS and Horovod paths are simply timed:
``src/distributed_worker.py:186-231``, ``horvod_pytorch.py:197-201``).
"""
import json
import math
import os
from dataclasses import dataclass, field

XGMI_LINK_GBPS = 153.0   # per link and direction; 7 links per MI355X (hardware sheet)
XGMI_LINKS = 7
RCCL_EFF = 0.4           # assumed: achieved / link-sum bandwidth of RCCL rings at these sizes
RCCL_ALPHA_US = 8.0      # assumed: fixed cost of one captured collective (launch, handshake)
RCCL_STEP_US = 1.5       # assumed: per ring step (one per peer for all-gather, two for all-reduce)


def bus_gbps(world: int) -> float:
    """Effective per-rank collective bandwidth (GB/s) with ``world`` ranks on one node."""
    return min(max(world - 1, 1), XGMI_LINKS) * XGMI_LINK_GBPS * RCCL_EFF


def allgather_us(world: int, bytes_per_rank: float) -> float:
    if world <= 1:
        return 0.0
    return (RCCL_ALPHA_US + (world - 1) * RCCL_STEP_US
            + (world - 1) * bytes_per_rank / (bus_gbps(world) * 1e3))


def allreduce_us(world: int, nbytes: float) -> float:
    if world <= 1:
        return 0.0
    return (RCCL_ALPHA_US + 2 * (world - 1) * RCCL_STEP_US
            + 2.0 * (world - 1) / world * nbytes / (bus_gbps(world) * 1e3))


@dataclass
class StepProfile:
    """Measured N = 1 numbers of one configuration (ms unless noted)."""
    full_ms: float           # the N = 1 step as bench.py runs it (unrolled one-graph step)
    seg_penalty_ms: float    # segmented minus the N > 1 one-graph step, world of one
    bwd_ms: float            # backward (the time a collective can hide behind)
    decode_us: dict = field(default_factory=dict)  # payloads -> decode + update us (top-k)
    # the N > 1 code path at world 1 minus full_ms: at N = 1 a one-bucket top-k step applies its
    # update in the encode's write pass and launches no decode (engine.enable_local_apply)
    n1_offset_ms: float = 0.0
    source: str = ""

    def decode_at(self, world: int) -> float:
        """Decode + update of ``world`` payloads (us): measured points, linear between them and
        beyond the last two."""
        if not self.decode_us:
            return 0.0
        pts = sorted((int(k), v) for k, v in self.decode_us.items())
        for (n0, t0), (n1, t1) in zip(pts, pts[1:]):
            if world <= n1:
                return t0 + (t1 - t0) * (world - n0) / (n1 - n0)
        (n0, t0), (n1, t1) = pts[-2], pts[-1]
        return t1 + (t1 - t0) * (world - n1) / (n1 - n0)


# N = 1 measurements, regenerated every round from that round's runs
# (tools/step_model_calibrate.py profiles/model/calib_rNN > parallel/n1_profiles.json; the raw
# bench lines and probe outputs stay under profiles/model/).  Keys (model, codec family, dtype);
# fp32, BASELINE batch per GPU.  In the package: every run (and the GPU box) reads the same file.
PROFILE_JSON = os.path.join(os.path.dirname(os.path.abspath(__file__)), "n1_profiles.json")


def _load_profiles(path: str = PROFILE_JSON) -> dict:
    try:
        with open(path) as f:
            raw = json.load(f)
    except (OSError, ValueError):
        return {}
    out = {}
    for key, p in raw.get("profiles", {}).items():
        m, fam, dt = key.split("/")
        out[(m, fam, dt)] = StepProfile(
            full_ms=p["full_ms"], seg_penalty_ms=p["seg_penalty_ms"], bwd_ms=p["bwd_ms"],
            decode_us=p.get("decode_us") or {}, n1_offset_ms=p.get("n1_offset_ms", 0.0),
            source=json.dumps(p.get("source", {}), sort_keys=True))
    return out


PROFILES = _load_profiles()

_MODEL_KEYS = {"vgg11": "vgg11", "vgg11_bn": "vgg11", "resnet50": "resnet50", "lenet": "lenet",
               "resnet50_imagenet": "resnet50_imagenet"}


def profile_for(model: str, codec_kind: str, dtype: str = "fp32"):
    """The measured profile of (model, codec family, compute dtype), or None."""
    key = _MODEL_KEYS.get((model or "").lower())
    fam = "topk" if codec_kind in ("topk", "topk_qsgd") else "dense"
    return PROFILES.get((key, fam, dtype)) if key else None


def predict(prof: StepProfile, world: int, codec_kind: str, payload_bytes_per_rank: float,
            dense_bytes: float, splits: int = 1) -> dict:
    """Predicted ms per step for ``full`` and ``segmented`` at ``world`` ranks.  ``dense_bytes``:
    the all-reduce's bytes (the wire dtype's: 2 per element for fp16 / bf16 codecs)."""
    if codec_kind in ("none", "fp16", "bf16"):
        comm = allreduce_us(world, dense_bytes)
    else:
        comm = allgather_us(world, payload_bytes_per_rank)
    base = prof.full_ms + (prof.n1_offset_ms if world > 1 else 0.0)
    decode_delta = prof.decode_at(world) - prof.decode_at(1) if prof.decode_us else 0.0
    full = base + (comm + decode_delta) / 1e3
    s = max(1, splits)
    tail = comm / (s + 1)                                     # the last split's collective
    spill = max(0.0, comm * s / (s + 1) - prof.bwd_ms * 1e3)  # more than backward can hide
    # (a segmented step never applies locally: at world 1 it pays the N > 1 path's offset too)
    seg = (prof.full_ms + prof.n1_offset_ms + prof.seg_penalty_ms
           + (tail + spill + decode_delta) / 1e3)
    return {"full": round(full, 4), "segmented": round(seg, 4), "comm_us": round(comm, 2),
            "decode_delta_us": round(decode_delta, 2)}


def overlap_splits(payload_bytes: float, max_splits: int, bytes_per_split: float) -> int:
    return int(min(max_splits, max(1, math.ceil(payload_bytes / bytes_per_split))))
