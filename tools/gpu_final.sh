#!/bin/bash
# end-of-session validation: all GPU tests, smoke, every BASELINE preset, VGG-11 profile
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
PRESETS="vgg11 lenet resnet50_cifar resnet50_imagenet" bash tools/gpu_validate.sh || exit 1
mkdir -p gpurun_out/prof24
export TMPDIR=/tmp EWDML_PROF_GAP=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_vgg -o run -- python3 bench.py --steps 20 --warmup 6 > gpurun_out/prof24/vgg.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof24/vgg.log; exit 1; }
python3 tools/prof_summarize.py /tmp/p_vgg gpurun_out/prof24/vgg_summary.txt --steps 20 > /dev/null || exit 1
head -1 gpurun_out/prof24/vgg_summary.txt
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --preset resnet50_cifar --steps 10 --warmup 6 > gpurun_out/prof24/r50c.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof24/r50c.log; exit 1; }
python3 tools/prof_summarize.py /tmp/p_r50 gpurun_out/prof24/r50c_summary.txt --steps 10 > /dev/null || exit 1
head -1 gpurun_out/prof24/r50c_summary.txt
