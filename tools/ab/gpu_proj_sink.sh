# projection-shortcut gradient sink: ResNet tests, then A/B against identity-only sinks
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/kernels/test_conv_f32.py -k "sink or resnet" tests/kernels/test_conv.py tests/kernels/test_nn_kernels.py > gpurun_out/sink_tests.log 2>&1
rc=$?; grep -E "^E |FAIL|passed|failed" gpurun_out/sink_tests.log | tail -30
[ $rc -gt 1 ] && exit 1
bash tools/gpurun_suite.sh ab 2 "base|EWDML_PROJ_SINK=0|--preset resnet50_cifar --no-extras" "sink||--preset resnet50_cifar --no-extras" "ibase|EWDML_PROJ_SINK=0|--preset resnet50_imagenet --no-extras" "isink||--preset resnet50_imagenet --no-extras"
