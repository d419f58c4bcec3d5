#!/bin/bash
# MIOpen solver A/B: disable the asm NHWC igemm bwd-data / wrw solvers (they need a zero-fill and
# an fp32->bf16 cast kernel per call) and let MIOpen find pick another solver
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -f gpurun_out/ab.log
W=MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_WRW_GTC_XDLOPS_NHWC=0
B=MIOPEN_DEBUG_CONV_IMPLICIT_GEMM_ASM_BWD_GTC_XDLOPS_NHWC=0
bash tools/ab.sh 2 "base|EWDML_X=0|" "nowrw|$W|" "nobwd|$B|" "none|$W $B|"
