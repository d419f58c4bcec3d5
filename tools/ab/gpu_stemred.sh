#!/bin/bash
# conv2's split-K reduction in the stem's reduction launch: tests, A/B, trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_conv_f32.py tests/e2e/test_gpu_train.py -q --timeout 300 \
    --timeout-method thread -k "deferred or rides or vgg11 or stem or unrolled or graph_modes or lazy" > gpurun_out/stemred_tests.log 2>&1
rc=$?; tail -3 gpurun_out/stemred_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 3 "ride||--no-extras" "noride|EWDML_BN_FIN_RIDE=0|--no-extras" || exit 1
bash tools/gpurun_suite.sh prof vgg_stemred "--no-extras" > /dev/null || exit 1
grep -E "reduce|per step" gpurun_out/prof_vgg_stemred.txt | head -6
