# ResNet-50 CIFAR step traces with / without the lazy 1x1 BN operand
set -o pipefail
bash tools/gpurun_suite.sh prof r50_lz1 "--preset resnet50_cifar --steps 10" > /dev/null && \
EWDML_LAZY_1X1=0 bash tools/gpurun_suite.sh prof r50_mat "--preset resnet50_cifar --steps 10" > /dev/null
