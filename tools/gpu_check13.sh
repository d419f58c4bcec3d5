#!/bin/bash
# RCCL-process-group bench test, then bucket-size A/B on VGG-11
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/e2e/test_gpu_train.py -x -q -k rccl --timeout 300 --timeout-method thread > gpurun_out/rccl_test.log 2>&1 || { tail -60 gpurun_out/rccl_test.log; exit 1; }
tail -2 gpurun_out/rccl_test.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "b64|EWDML_X=0|" "b24|EWDML_X=0|--bucket-mb 24" "b12|EWDML_X=0|--bucket-mb 12"
