#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/kernels/test_head_tail.py -q --timeout 120 --timeout-method thread > gpurun_out/tail_tests.log 2>&1
rc=$?; tail -1 gpurun_out/tail_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh prof vgg_tail "--no-extras" > /dev/null || exit 1
grep -E "k_tail|per step" gpurun_out/prof_vgg_tail.txt | head -4
bash tools/gpurun_suite.sh ab 3 "tail||--no-extras" "perlinear|EWDML_HEAD_TAIL=0|--no-extras" || exit 1
