#!/bin/bash
# top-k pass-0 histogram with bank-spread LDS copies: codec tests, VGG-11 trace, bench
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/hist
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/kernels/test_hip_codecs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/hist/tests.log 2>&1 || { tail -40 gpurun_out/hist/tests.log; exit 1; }
tail -1 gpurun_out/hist/tests.log
EWDML_PROF_GAP=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/h1 -o run -- python3 bench.py --steps 20 --warmup 6 > gpurun_out/hist/p.log 2>&1 || { tail -30 gpurun_out/hist/p.log; exit 1; }
python3 tools/prof_summarize.py /tmp/h1 gpurun_out/hist/vgg_summary.txt --steps 20 > /dev/null || exit 1
head -1 gpurun_out/hist/vgg_summary.txt; grep topk gpurun_out/hist/vgg_summary.txt | head -12
for i in 1 2; do timeout -k 10 300 python bench.py > gpurun_out/hist/b$i.json 2>gpurun_out/hist/err.log || { tail -20 gpurun_out/hist/err.log; exit 1; }; cut -c1-190 gpurun_out/hist/b$i.json; done
