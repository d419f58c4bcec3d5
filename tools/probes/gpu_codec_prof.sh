#!/bin/bash
# Codec kernel tests, then a kernel-trace profile of the VGG-11 fp32 top-k step (codec kernels and
# the bench value).  Run through gpurun from the repo root.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_hip_codecs.py -x -q --timeout 120 \
    --timeout-method thread > gpurun_out/codec_tests.log 2>&1 || { tail -30 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
bash tools/gpurun_suite.sh prof pk_vgg "--no-extras --steps 20 ${PROF_ARGS:-}" > gpurun_out/combo_prof.txt 2>&1 \
    || { tail -20 gpurun_out/combo_prof.txt; exit 1; }
head -1 gpurun_out/prof_pk_vgg.txt
grep -E "k_pk|k_topk" gpurun_out/prof_pk_vgg.txt | grep -v -- "->" | head -6
grep "^{" gpurun_out/combo_prof.txt | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print('value', d['value'], d['codec_health'])"
