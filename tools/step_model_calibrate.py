"""Regenerate the step model's N = 1 profiles (parallel/n1_profiles.json) from a directory of
round measurements (tools/ab/calib_r06.sh writes one: gpurun_out/calib/, committed as
profiles/model/calib_r06/):

    python tools/step_model_calibrate.py profiles/model/calib_r06 \
        > efficient-workers-in-distributed-machine-learning_amd/parallel/n1_profiles.json

* presets.jsonl        -- bench.py lines of the BASELINE presets, top-k and dense (full_ms: the
                          N = 1 step as bench runs it);
* no_local_apply.jsonl -- the top-k presets with EWDML_LOCAL_APPLY=0: the N > 1 code path at world
                          1 (encode, all-gather of one payload, decode) -> n1_offset_ms;
* segmented.jsonl      -- with the real communicator (EWDML_FORCE_PG=1): --hip-graph full
                          --graph-unroll 1 and segmented -> seg_penalty_ms (segmented minus the
                          N > 1 one-graph step bench would run);
* decode_<model>.json  -- tools/probes/decode_probe.py: decode + update of 1/2/4/8 payloads.

Backward times (what a segmented step's collectives can hide behind) are not separable from one
bench line; they stay the trace-based estimates below."""
import json
import os
import sys

BWD_MS = {"vgg11": (0.78, "trace estimate (profiles/vgg11_bs128_fp32_current_graph.txt)"),
          "lenet": (0.037, "trace estimate (k_ln_fc_bwd + k_ln_conv_bwd, profiles/lenet_*)"),
          "resnet50": (9.0, "trace estimate (profiles/resnet50_cifar_bs128_fp32_graph.txt)"),
          "resnet50_imagenet": (14.5, "trace estimate (profiles/resnet50_imagenet_bs64_fp32_graph.txt)")}
MODEL_KEY = {"vgg11_bn": "vgg11", "LeNet": "lenet", "ResNet50": "resnet50",
             "resnet50_imagenet": "resnet50_imagenet"}


def _lines(path):
    if not os.path.exists(path):
        return []
    with open(path) as f:
        return [json.loads(l) for l in f if l.startswith("{")]


def _fam(rec):
    return "dense" if rec["config"]["codec"] in ("none", "fp16", "bf16") else "topk"


def main(d):
    prof = {}
    for r in _lines(os.path.join(d, "presets.jsonl")):
        m = MODEL_KEY[r["config"]["model"]]
        key = f"{m}/{_fam(r)}/{r['dtype']}"
        prof[key] = {"full_ms": r["ms_per_step"], "n1_offset_ms": 0.0,
                     "seg_penalty_ms": None, "bwd_ms": BWD_MS[m][0],
                     "decode_us": {}, "source": {"full_ms": "presets.jsonl",
                                                 "bwd_ms": BWD_MS[m][1]}}
    for r in _lines(os.path.join(d, "no_local_apply.jsonl")):
        m = MODEL_KEY[r["config"]["model"]]
        p = prof.get(f"{m}/{_fam(r)}/{r['dtype']}")
        if p is not None:
            # (0 where both runs took the same path: several buckets never apply locally)
            p["n1_offset_ms"] = round(max(0.0, r["ms_per_step"] - p["full_ms"]), 4)
            p["source"]["n1_offset_ms"] = "no_local_apply.jsonl minus presets.jsonl"
    seg = {}
    for r in _lines(os.path.join(d, "segmented.jsonl")):
        m = MODEL_KEY[r["config"]["model"]]
        seg.setdefault(f"{m}/{_fam(r)}/{r['dtype']}", {})[r["config"]["hip_graph"]] = r
    for key, v in seg.items():
        p = prof.get(key)
        if p is None or "segmented" not in v:
            continue
        # relative to the N > 1 one-graph step bench runs (unrolled graphs, decode launch)
        p["seg_penalty_ms"] = round(v["segmented"]["ms_per_step"] - p["full_ms"]
                                    - p["n1_offset_ms"], 4)
        p["source"]["seg_penalty_ms"] = "segmented.jsonl (real communicator, world 1)"
    for key, p in prof.items():
        m, fam, _ = key.split("/")
        dec = os.path.join(d, f"decode_{m}.json")
        if fam == "topk" and os.path.exists(dec):
            with open(dec) as f:
                p["decode_us"] = json.load(f)["decode_us"]
            p["source"]["decode_us"] = os.path.basename(dec)
        if p["seg_penalty_ms"] is None:  # unmeasured: the same model's dense penalty, else VGG's
            other = prof.get(f"{m}/dense/fp32", {}).get("seg_penalty_ms")
            p["seg_penalty_ms"] = other if other is not None else 0.1
            p["source"]["seg_penalty_ms"] = ("assumed: the model's dense penalty" if other
                                             is not None else "assumed")
    json.dump({"measured": os.path.normpath(d), "profiles": prof}, sys.stdout, indent=1,
              sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/model/calib_r06")
