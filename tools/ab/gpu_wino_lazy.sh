#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpurun_suite.sh ab 3 "wlazy||--no-extras" "wplain|EWDML_WINO_LAZY_BWD=0|--no-extras" || exit 1
