# Lazy BN + ReLU into ResNet's 1x1 conv3 (conv_f32.hip CfLz): tests, then an interleaved A/B on
# both ResNet-50 presets.
set -o pipefail
TESTS_ARGS="tests/kernels/test_conv_f32.py" TESTS_K="lazy or resnet or projection or 1x1" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 2 "lz1||--preset resnet50_cifar --no-extras" "mat|EWDML_LAZY_1X1=0|--preset resnet50_cifar --no-extras" && \
bash tools/gpurun_suite.sh ab 2 "lz1i||--preset resnet50_imagenet --no-extras" "mati|EWDML_LAZY_1X1=0|--preset resnet50_imagenet --no-extras"
