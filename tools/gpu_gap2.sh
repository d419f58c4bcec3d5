#!/bin/bash
# VGG-11 mid-backward idle gap: eager vs split graph vs packet-capture off
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/gap2
export TMPDIR=/tmp EWDML_PROF_GAP=1
run() {  # name, env assignment or '', bench args
  local n=$1; shift
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/$n -o run -- python3 bench.py --steps 20 --warmup 6 "$@" > gpurun_out/gap2/$n.log 2>&1 || { tail -30 gpurun_out/gap2/$n.log; return 1; }
  python3 tools/prof_summarize.py /tmp/$n gpurun_out/gap2/${n}_summary.txt --steps 20 > /dev/null || return 1
  head -1 gpurun_out/gap2/${n}_summary.txt
}
run eager --hip-graph off && run split --hip-graph split && \
DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 run nopc && HIP_FORCE_DEV_KERNARG=1 run devk
