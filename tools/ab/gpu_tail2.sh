#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpurun_suite.sh prof vgg_tail "--no-extras" > /dev/null || exit 1
grep -E "k_tail|k_head|k_ce|per step" gpurun_out/prof_vgg_tail.txt | head -12
