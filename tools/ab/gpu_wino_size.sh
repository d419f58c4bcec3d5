# Winograd tile "size" default (m = 4 with >= 2048 output tiles) vs m = 2: conv tests, A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_conv_f32.py tests/e2e/test_gpu_train.py > gpurun_out/wino_tests.log 2>&1 || { grep -E "FAIL|Error|assert|passed|failed" gpurun_out/wino_tests.log | tail -30; exit 1; }
tail -1 gpurun_out/wino_tests.log
bash tools/gpurun_suite.sh ab 2 "size||--preset resnet50_cifar --no-extras" "m2|EWDML_WINO_TILE=2|--preset resnet50_cifar --no-extras" "isize||--preset resnet50_imagenet --no-extras" "im2|EWDML_WINO_TILE=2|--preset resnet50_imagenet --no-extras" "vsize||--no-extras" "vm2|EWDML_WINO_TILE=2|--no-extras"
