#!/bin/bash
# MFMA conv: numerics tests, per-layer timings vs MIOpen, bench A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv.py -x -v --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -60 gpurun_out/conv_tests.log; exit 1; }
tail -3 gpurun_out/conv_tests.log
timeout -k 10 300 python tools/conv_probe.py > gpurun_out/conv_probe.log 2>&1 || { tail -30 gpurun_out/conv_probe.log; exit 1; }
cat gpurun_out/conv_probe.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "hipconv|EWDML_CONV=hip|" "miopen|EWDML_CONV=miopen|"
