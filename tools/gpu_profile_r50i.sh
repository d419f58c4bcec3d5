#!/bin/bash
# kernel-trace profile of the ResNet-50 224x224 bench step
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof22
export TMPDIR=/tmp EWDML_PROF_GAP=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_r50i -o run -- python3 bench.py --preset resnet50_imagenet --steps 10 --warmup 6 > gpurun_out/prof22/r50i.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof22/r50i.log; exit 1; }
python3 tools/prof_summarize.py /tmp/p_r50i gpurun_out/prof22/r50i_summary.txt --steps 10 > /dev/null || exit 1
head -45 gpurun_out/prof22/r50i_summary.txt | cut -c1-150
