#!/bin/bash
# In-hist0 select for tensors with few candidates: codec tests, then LeNet / VGG-11 bench pairs
# against the candidate-pass select (EWDML_TOPK_INLINE=0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_hip_codecs.py -q -x --timeout 120 --timeout-method thread \
    > gpurun_out/codec_tests.log 2>&1
rc=$?; tail -3 gpurun_out/codec_tests.log; grep -E "^E |FAILED" gpurun_out/codec_tests.log | head -12
[ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "lenet_inline||--preset lenet --no-extras" "lenet_passes|EWDML_TOPK_INLINE=0|--preset lenet --no-extras" \
    "vgg_inline||--no-extras" "vgg_passes|EWDML_TOPK_INLINE=0|--no-extras" || exit 1
timeout -k 10 120 python -u tools/probes/launch_floor.py || exit 1
