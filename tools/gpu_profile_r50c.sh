#!/bin/bash
# kernel-trace profile of the ResNet-50 CIFAR bench step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof25
export TMPDIR=/tmp EWDML_PROF_GAP=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_r50 -o run -- python3 bench.py --preset resnet50_cifar --steps 10 --warmup 6 > gpurun_out/prof25/r50c.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof25/r50c.log; exit 1; }
python3 tools/prof_summarize.py /tmp/p_r50 gpurun_out/prof25/r50c_summary.txt --steps 10 > /dev/null || exit 1
head -40 gpurun_out/prof25/r50c_summary.txt | cut -c1-120
