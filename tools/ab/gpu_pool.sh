# 3x3/s2 max pool: kernel test vs torch, ResNet-50 224 bench
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_nn_kernels.py > gpurun_out/nn_tests.log 2>&1 || { tail -40 gpurun_out/nn_tests.log; exit 1; }
tail -1 gpurun_out/nn_tests.log
bash tools/gpurun_suite.sh bench "--preset resnet50_imagenet --no-extras" "--preset resnet50_imagenet --no-extras"
