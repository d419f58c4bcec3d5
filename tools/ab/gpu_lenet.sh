#!/bin/bash
# Fused LeNet step: kernel tests, the LeNet accuracy tests, bench A/B against the module path
# (EWDML_LENET_FUSED=0), kernel trace of the fused step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_lenet_fused.py -v --timeout 120 --timeout-method thread \
    > gpurun_out/lenet_tests.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/lenet_tests.log | tail -12
[ $rc -eq 0 ] || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u bench.py --preset lenet --no-extras > gpurun_out/lenet_bench$i.log 2>&1 || exit 1
  tail -1 gpurun_out/lenet_bench$i.log | cut -c1-220
  EWDML_LENET_FUSED=0 timeout -k 10 300 python -u bench.py --preset lenet --no-extras > gpurun_out/lenet_bench_mod$i.log 2>&1 || exit 1
  tail -1 gpurun_out/lenet_bench_mod$i.log | cut -c1-220
done
bash tools/gpurun_suite.sh prof lenet_fused "--preset lenet --no-extras" || exit 1
timeout -k 10 900 python -u -m pytest tests/e2e/test_gpu_accuracy.py -v --timeout 300 --timeout-method thread -k lenet \
    > gpurun_out/lenet_acc.log 2>&1
grep -E "PASSED|FAILED|Error|passed|failed" gpurun_out/lenet_acc.log | tail -10
