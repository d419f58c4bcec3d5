#!/bin/bash
# Predictive-encode hist0 held to 4 / 5 waves per SIMD (EWDML_PK_H0_WPE, two-half DGC staging) and
# the 1024-thread forward BN finalize (EWDML_BN_FIN_WIDE): codec tests per variant, then A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
for w in 4 5; do
  EWDML_PK_H0_WPE=$w timeout -k 10 300 python -u -m pytest tests/kernels/test_hip_codecs.py -q --timeout 120 \
      --timeout-method thread -k "dgc or predictive or error_feedback" > gpurun_out/h0_tests_$w.log 2>&1
  rc=$?; tail -1 gpurun_out/h0_tests_$w.log; [ $rc -eq 0 ] || exit 1
done
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv_f32.py -q --timeout 120 --timeout-method thread \
    -k "vgg11 or bn_statistics" > gpurun_out/finwide_tests.log 2>&1
rc=$?; tail -1 gpurun_out/finwide_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh ab 2 "base|EWDML_BN_FIN_WIDE=0|--no-extras" "wide||--no-extras" \
    "wide_h4|EWDML_PK_H0_WPE=4|--no-extras" "wide_h5|EWDML_PK_H0_WPE=5|--no-extras" || exit 1
EWDML_PK_H0_WPE=4 bash tools/gpurun_suite.sh prof vgg_h4 "--no-extras" > /dev/null || exit 1
grep -E "hist0|fwd_finalize|per step" gpurun_out/prof_vgg_h4.txt | head -5
