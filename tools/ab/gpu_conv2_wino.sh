#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpurun_suite.sh ab 3 "direct||--no-extras" "wino64|EWDML_WINO_MIN_C=64|--no-extras" "wino64m2|EWDML_WINO_MIN_C=64 EWDML_WINO_M4_MIN_TILES=4096|--no-extras" || exit 1
