#!/bin/bash
# 8-way split small-map forward: tests, standalone timing, step trace, bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 120 --timeout-method thread \
    -k "smallmap or vgg11" > gpurun_out/sm8_tests.log 2>&1
rc=$?; tail -1 gpurun_out/sm8_tests.log; grep -E "^E |FAILED" gpurun_out/sm8_tests.log | head -5
[ $rc -eq 0 ] || exit 1
timeout -k 10 120 python -u tools/probes/sm_probe.py 2>&1 | grep -v amdgpu.ids || exit 1
bash tools/gpurun_suite.sh prof vgg_sm8 "--no-extras" > /dev/null || exit 1
grep -E "k_sm_|per step" gpurun_out/prof_vgg_sm8.txt | head -5
bash tools/gpurun_suite.sh ab 2 "vgg||--no-extras" || exit 1
