"""Write profiles/model/step_model.md: the N > 1 step model's constants, N = 1 profiles and
predictions for the BASELINE presets (python tools/step_model_table.py > profiles/model/step_model.md)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from ewdml.parallel import step_model as sm  # noqa: E402
from ewdml.parallel.engine import plan_graph_mode  # noqa: E402

print("# N > 1 step model (`parallel/step_model.py`): constants, sources, predictions\n")
print("The exchange has never run at N > 1 (one-GPU development pool; the driver's 8-GPU SCALE run")
print("is the first).  These predictions are what that run is checked against; `bench.py` prints")
print("`predicted_ms_per_step` for the graph mode it ran.  Regenerate: `python tools/step_model_table.py`.\n")
print("## Constants\n")
print("| constant | value | source |\n|---|---|---|")
print(f"| xGMI link bandwidth | {sm.XGMI_LINK_GBPS} GB/s per link and direction, {sm.XGMI_LINKS} links "
      "per GPU | MI355X hardware sheet (one link to each peer in the 8-GPU mesh) |")
print(f"| RCCL efficiency | {sm.RCCL_EFF} of the link sum | **assumed** (typical ring bus bandwidth "
      "on 8-GPU xGMI meshes); replace from SCALE |")
print(f"| collective latency | {sm.RCCL_ALPHA_US} us + {sm.RCCL_STEP_US} us per ring step | "
      "**assumed**; replace from SCALE |")
print("\n## N = 1 profiles (fp32, batch 128 per GPU)\n")
print("| model, codec family | full step ms | segmented - full ms | backward ms | decode us "
      "(payloads) | source |\n|---|---|---|---|---|---|")
for (m, f), p in sm.PROFILES.items():
    print(f"| {m}, {f} | {p.full_ms:.4f} | {p.seg_penalty_ms:.4f} | {p.bwd_ms} | "
          f"{p.decode_us or '-'} | {p.source} |")
print("\n## Predictions (ms per step; the mode `--hip-graph auto` picks marked *)\n")
print("| config | N | wire bytes/rank | collective us | full | segmented |\n|---|---|---|---|---|---|")
cfgs = [("VGG11 top-1% + QSGD-8", "VGG11", "topk_qsgd", 9756426),
        ("VGG11 dense fp32", "VGG11", "none", 9756426),
        ("ResNet50 CIFAR top-1% + QSGD-8", "ResNet50", "topk_qsgd", 23520842),
        ("ResNet50 CIFAR dense fp32", "ResNet50", "none", 23520842)]
for name, model, codec, n in cfgs:
    for w in (1, 2, 4, 8):
        p = plan_graph_mode(w, "rccl-stream" if w > 1 else "local", codec, n, model=model,
                            bucket_bytes=64 << 20)
        pr = p["predicted_ms"]
        f = f"{pr['full']:.4f}" + ("*" if p["mode"] == "full" else "")
        s = f"{pr['segmented']:.4f}" + ("*" if p["mode"] == "segmented" else "")
        print(f"| {name} | {w} | {p['wire_bytes']} | {pr['comm_us']} | {f} | {s} |")
