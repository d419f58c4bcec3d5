#!/bin/bash
# Deferred Winograd transform riding in the direct conv's backward-data GEMM: tests, A/B, trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 200 --timeout-method thread \
    -k "deferred or rides or vgg11 or resnet18 or backward" > gpurun_out/woride_tests.log 2>&1
rc=$?; tail -3 gpurun_out/woride_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 3 "ride||--no-extras" "noride|EWDML_BN_FIN_RIDE=0|--no-extras" || exit 1
bash tools/gpurun_suite.sh prof vgg_woride "--no-extras" > /dev/null || exit 1
grep -E "wgrad_out|per step|k_cf_gemm<1, 128, 64" gpurun_out/prof_vgg_woride.txt | head -8
