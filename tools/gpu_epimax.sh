#!/bin/bash
# size threshold of the conv epilogue fusions (EWDML_EPI_MAX elements), ResNet-50 / VGG-11
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
bash tools/ab.sh 1 "r50c_0|EWDML_EPI_MAX=0|--preset resnet50_cifar" "r50c_4M|EWDML_EPI_MAX=4194304|--preset resnet50_cifar" "r50c_8M|EWDML_EPI_MAX=8388608|--preset resnet50_cifar" "r50c_16M|EWDML_EPI_MAX=16777216|--preset resnet50_cifar" "r50c_inf|EWDML_EPI_MAX=1000000000|--preset resnet50_cifar" "vgg_0|EWDML_EPI_MAX=0|" "vgg_8M||" "r50i_0|EWDML_EPI_MAX=0|--preset resnet50_imagenet" "r50i_8M||--preset resnet50_imagenet"
