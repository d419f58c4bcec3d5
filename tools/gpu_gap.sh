#!/bin/bash
# where does the ~55 us mid-backward idle gap of the VGG-11 step come from?
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gap
export TMPDIR=/tmp EWDML_PROF_GAP=1
timeout -k 10 300 python bench.py > gpurun_out/gap/base.json 2>&1 || { tail -20 gpurun_out/gap/base.json; exit 1; }
timeout -k 10 300 python bench.py --no-overlap > gpurun_out/gap/noov.json 2>&1 || { tail -20 gpurun_out/gap/noov.json; exit 1; }
tail -1 gpurun_out/gap/base.json | cut -c1-200; tail -1 gpurun_out/gap/noov.json | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d /tmp/g1 -o run -- python3 bench.py --steps 20 --warmup 6 > gpurun_out/gap/p1.log 2>&1 || { tail -30 gpurun_out/gap/p1.log; exit 1; }
python3 tools/prof_summarize.py /tmp/g1 gpurun_out/gap/base_summary.txt --steps 20 > /dev/null || exit 1
find /tmp/g1 -name "*memory_copy*" -exec cp {} gpurun_out/gap/ \;
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/g2 -o run -- python3 bench.py --steps 20 --warmup 6 --no-overlap > gpurun_out/gap/p2.log 2>&1 || { tail -30 gpurun_out/gap/p2.log; exit 1; }
python3 tools/prof_summarize.py /tmp/g2 gpurun_out/gap/noov_summary.txt --steps 20 > /dev/null || exit 1
head -1 gpurun_out/gap/base_summary.txt gpurun_out/gap/noov_summary.txt
