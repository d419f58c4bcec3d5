# our stride-2 fp32 kernels vs MIOpen at the round-6 kernels (EWDML_CONV_S2)
set -o pipefail
bash tools/gpurun_suite.sh ab 2 "s2|EWDML_CONV_S2=1|--preset resnet50_cifar --no-extras" "miopen||--preset resnet50_cifar --no-extras" \
  "s2i|EWDML_CONV_S2=1|--preset resnet50_imagenet --no-extras" "miopeni||--preset resnet50_imagenet --no-extras"
