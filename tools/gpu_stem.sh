#!/bin/bash
# stem conv kernels: conv tests (incl. VGG / ResNet steps vs MIOpen), per-layer probe, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/kernels/test_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/stem_tests.log 2>&1 || { tail -50 gpurun_out/stem_tests.log; exit 1; }
tail -1 gpurun_out/stem_tests.log
timeout -k 10 300 python -u tools/conv_probe.py > gpurun_out/conv_probe_stem.log 2>&1 || { tail -20 gpurun_out/conv_probe_stem.log; exit 1; }
head -4 gpurun_out/conv_probe_stem.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg||" "r50c||--preset resnet50_cifar"
