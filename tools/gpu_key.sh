#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/e2e tests/kernels/test_hip_codecs.py -x -q --timeout 200 --timeout-method thread > gpurun_out/key_tests.log 2>&1 || { tail -60 gpurun_out/key_tests.log; exit 1; }
tail -1 gpurun_out/key_tests.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg|EWDML_X=0|"
