# 64x256 weight-gradient tiles: conv tests vs float64, ResNet-50 CIFAR A/B (EWDML_CF_WIDE=0/1), VGG check
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_conv_f32.py > gpurun_out/conv_tests.log 2>&1 || { tail -40 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
bash tools/gpurun_suite.sh ab 2 "wide|EWDML_CF_WIDE=1|--preset resnet50_cifar --no-extras" "narrow|EWDML_CF_WIDE=0|--preset resnet50_cifar --no-extras" "vgg_wide|EWDML_CF_WIDE=1|--no-extras" "vgg_narrow|EWDML_CF_WIDE=0|--no-extras"
