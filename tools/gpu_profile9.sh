#!/bin/bash
# kernel profile of the current default VGG-11 bench (MFMA convs)
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof9
export TMPDIR=/tmp EWDML_PROF_GAP=1
timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_vgg -o run -- python3 bench.py --steps 20 --warmup 6 > gpurun_out/prof9/vgg.log 2>&1 || { echo "prof failed"; tail -30 gpurun_out/prof9/vgg.log; exit 1; }
python3 tools/prof_summarize.py /tmp/p_vgg gpurun_out/prof9/vgg11_summary.txt --steps 20 > /dev/null || exit 1
head -50 gpurun_out/prof9/vgg11_summary.txt
