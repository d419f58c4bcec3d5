#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest gpu rc=$rc"; tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|error|assert" gpurun_out/pytest_gpu.log | head -30; exit 1; }
rm -f gpurun_out/ab.log
bash tools/ab.sh 3 "bf16p_topk|EWDML_X=0|" "fp32p_topk|EWDML_X=0|--param-dtype fp32" "bf16p_dense|EWDML_X=0|--compress none" "fp32p_dense|EWDML_X=0|--compress none --param-dtype fp32"
