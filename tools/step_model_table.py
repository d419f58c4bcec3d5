"""Write profiles/model/step_model.md: the N > 1 step model's constants, N = 1 profiles and
predictions for the BASELINE presets (python tools/step_model_table.py > profiles/model/step_model.md)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ewdml.parallel import step_model as sm  # noqa: E402
from ewdml.parallel.engine import plan_graph_mode  # noqa: E402

print("# N > 1 step model (`parallel/step_model.py`): constants, sources, predictions\n")
print("The exchange has never run at N > 1 on this pool (one GPU per box).  These predictions are")
print("what a scaling run is checked against; `bench.py` prints `predicted_ms_per_step` for the graph")
print("mode it ran and, at N = 1, `model_error_n1`.  The N = 1 profiles are regenerated every round")
print("from that round's runs: `bash tools/ab/calib_r06.sh` (GPU) -> `profiles/model/calib_r06/` ->")
print("`python tools/step_model_calibrate.py profiles/model/calib_r06 > .../parallel/n1_profiles.json`;")
print("this file: `python tools/step_model_table.py > profiles/model/step_model.md`.\n")
print("## Constants\n")
print("| constant | value | source |\n|---|---|---|")
print(f"| xGMI link bandwidth | {sm.XGMI_LINK_GBPS} GB/s per link and direction, {sm.XGMI_LINKS} links "
      "per GPU | MI355X hardware sheet (one link to each peer in the 8-GPU mesh) |")
print(f"| RCCL efficiency | {sm.RCCL_EFF} of the link sum | **assumed** (typical ring bus bandwidth "
      "on 8-GPU xGMI meshes); replace from SCALE |")
print(f"| collective latency | {sm.RCCL_ALPHA_US} us + {sm.RCCL_STEP_US} us per ring step | "
      "**assumed**; replace from SCALE |")
print("\n## N = 1 profiles (fp32, BASELINE batch per GPU; `parallel/n1_profiles.json`)\n")
print("| model, codec family, dtype | full step ms | N > 1 path offset ms | segmented penalty ms | "
      "backward ms | decode us (payloads) | sources |\n|---|---|---|---|---|---|---|")
for (m, f, dt), p in sorted(sm.PROFILES.items()):
    print(f"| {m}, {f}, {dt} | {p.full_ms:.4f} | {p.n1_offset_ms:.4f} | {p.seg_penalty_ms:.4f} | "
          f"{p.bwd_ms} | {p.decode_us or '-'} | `{p.source}` |")
print("\n## Predictions (ms per step; the mode `--hip-graph auto` picks marked *)\n")
print("| config | N | wire bytes/rank | collective us | full | segmented |\n|---|---|---|---|---|---|")
cfgs = [("VGG11 top-1% + QSGD-8", "VGG11", "topk_qsgd", 9756426, 0.01, 8),
        ("VGG11 dense fp32", "VGG11", "none", 9756426, 0.01, 8),
        ("LeNet top-1% + QSGD-8", "LeNet", "topk_qsgd", 431080, 0.01, 8),
        ("LeNet dense fp32", "LeNet", "none", 431080, 0.01, 8),
        ("ResNet50 CIFAR top-1% + QSGD-8", "ResNet50", "topk_qsgd", 23520842, 0.01, 8),
        ("ResNet50 CIFAR dense fp32", "ResNet50", "none", 23520842, 0.01, 8),
        ("ResNet50 224px top-0.1% + QSGD-4", "resnet50_imagenet", "topk_qsgd", 25557032, 0.001,
         4),
        ("ResNet50 224px dense fp32", "resnet50_imagenet", "none", 25557032, 0.001, 4)]
for name, model, codec, n, ratio, bits in cfgs:
    for w in (1, 2, 4, 8):
        p = plan_graph_mode(w, "rccl-stream" if w > 1 else "local", codec, n, model=model,
                            bucket_bytes=64 << 20, topk_ratio=ratio, bits=bits)
        pr = p["predicted_ms"]
        f = f"{pr['full']:.4f}" + ("*" if p["mode"] == "full" else "")
        s = f"{pr['segmented']:.4f}" + ("*" if p["mode"] == "segmented" else "")
        print(f"| {name} | {w} | {p['wire_bytes']} | {pr['comm_us']} | {f} | {s} |")
