# Winograd F(4x4) for ResNet-50's 64-channel 3x3 layers (EWDML_WINO_M4_MAX_C=64) vs direct GEMM
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpurun_suite.sh ab 2 "base||--preset resnet50_cifar --no-extras" "c64|EWDML_WINO_M4_MAX_C=64|--preset resnet50_cifar --no-extras" "ibase||--preset resnet50_imagenet --no-extras" "ic64|EWDML_WINO_M4_MAX_C=64|--preset resnet50_imagenet --no-extras"
