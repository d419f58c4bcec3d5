#!/bin/bash
# probes: graph launch cost, per-layer conv/GEMM timings, MIOpen find-mode A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out


timeout -k 10 300 python tools/conv_probe.py > gpurun_out/conv_probe.log 2>&1 || { tail -20 gpurun_out/conv_probe.log; exit 1; }
cat gpurun_out/conv_probe.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 1 "base|EWDML_X=0|" "find_normal|MIOPEN_FIND_MODE=1|"
