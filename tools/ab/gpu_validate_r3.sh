# round-3 end validation: full GPU suite (log kept), smoke, default bench (+ extras), presets
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
bash tools/gpurun_suite.sh bench "" "--preset lenet --no-extras" "--preset resnet50_cifar --no-extras" "--preset resnet50_imagenet --no-extras" "--preset resnet50_cifar --no-extras --amp bf16" "--preset resnet50_imagenet --no-extras --amp bf16"
