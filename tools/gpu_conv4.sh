#!/bin/bash
# LDS-DMA conv kernels: numerics (both paths), then A/B
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
#EWDML_CONV_DMA=1 timeout -k 10 300 python -u -m pytest tests/kernels/test_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests_dma.log 2>&1 || { tail -60 gpurun_out/conv_tests_dma.log; exit 1; }
#tail -1 gpurun_out/conv_tests_dma.log
#timeout -k 10 300 python -u -m pytest tests/kernels/test_conv.py tests/kernels/test_nn_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -60 gpurun_out/conv_tests.log; exit 1; }
#tail -1 gpurun_out/conv_tests.log
EWDML_CONV_DMA=1 timeout -k 10 300 python tools/conv_probe.py > gpurun_out/conv_probe_dma.log 2>&1 || { tail -30 gpurun_out/conv_probe_dma.log; exit 1; }
cat gpurun_out/conv_probe_dma.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg_dma|EWDML_CONV_DMA=1|" "vgg_kg|EWDML_CONV_DMA=0|" "r50c_dma|EWDML_CONV_DMA=1|--preset resnet50_cifar" "r50c_kg|EWDML_CONV_DMA=0|--preset resnet50_cifar"
