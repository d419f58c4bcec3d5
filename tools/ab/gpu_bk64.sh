#!/bin/bash
# 64-deep k-steps in the 2x2-map GEMMs: kernel tests, standalone timing, a VGG-11 bench pair.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/kernels/test_conv_f32.py -v --timeout 120 --timeout-method thread \
    -k "smallmap or vgg11 or lazy" > gpurun_out/bk64_tests.log 2>&1
rc=$?; grep -E "FAILED|Error:|passed|failed" gpurun_out/bk64_tests.log | tail -15
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 1
timeout -k 10 120 python -u tools/probes/sm_probe.py > gpurun_out/bk64_probe.log 2>&1 || exit 1
cat gpurun_out/bk64_probe.log
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --no-extras > gpurun_out/bk64_bench$i.log 2>&1 || exit 1
  tail -1 gpurun_out/bk64_bench$i.log | cut -c1-200
done
