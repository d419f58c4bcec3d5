#!/bin/bash
# Small-map kernels in the step with and without the lazy BN operands (EWDML_LAZY_BN=0): traces.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpurun_suite.sh prof vgg_lazy "--no-extras" > /dev/null || exit 1
EWDML_LAZY_BN=0 bash tools/gpurun_suite.sh prof vgg_nolazy "--no-extras" > /dev/null || exit 1
grep -E "k_sm_|per step" gpurun_out/prof_vgg_lazy.txt | head -6
grep -E "k_sm_|per step" gpurun_out/prof_vgg_nolazy.txt | head -6
