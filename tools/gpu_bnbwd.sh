#!/bin/bash
# fused head GEMM kernels: kernel + e2e tests, bench, kernel-trace profile of the VGG-11 step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof24
export TMPDIR=/tmp EWDML_PROF_GAP=1
timeout -k 10 300 python -u -m pytest tests/kernels/test_nn_kernels.py tests/kernels/test_make_batch.py tests/kernels/test_conv.py -x -q --timeout 120 --timeout-method thread > gpurun_out/prof24/tests.log 2>&1 || { tail -60 gpurun_out/prof24/tests.log; exit 1; }
tail -1 gpurun_out/prof24/tests.log
timeout -k 10 400 python -u -m pytest tests/e2e/test_gpu_train.py -x -q --timeout 200 --timeout-method thread > gpurun_out/prof24/e2e.log 2>&1 || { tail -60 gpurun_out/prof24/e2e.log; exit 1; }
tail -1 gpurun_out/prof24/e2e.log
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "vgg||" "r50c||--preset resnet50_cifar" "r50i||--preset resnet50_imagenet" || exit 1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_vgg -o run -- python3 bench.py --steps 20 --warmup 6 > gpurun_out/prof24/vgg.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof24/vgg.log; exit 1; }
python3 tools/prof_summarize.py /tmp/p_vgg gpurun_out/prof24/vgg_summary.txt --steps 20 > /dev/null || exit 1
head -1 gpurun_out/prof24/vgg_summary.txt
grep -E "head|ce_" gpurun_out/prof24/vgg_summary.txt | head -8
