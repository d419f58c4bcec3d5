#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpurun_suite.sh ab 3 "smlazy||--no-extras" "smplain|EWDML_SM_LAZY_BWD=0|--no-extras" || exit 1
EWDML_SM_LAZY_BWD=0 bash tools/gpurun_suite.sh prof vgg_smplain "--no-extras" > /dev/null || exit 1
grep -E "k_sm_|k_bn_bwd_apply|per step" gpurun_out/prof_vgg_smplain.txt | head -8
