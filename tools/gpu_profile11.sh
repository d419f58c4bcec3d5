#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof11
export TMPDIR=/tmp EWDML_PROF_GAP=1
for v in "fused:fused" "torch:torch"; do
  name=${v%%:*}; h=${v#*:}
  EWDML_HEAD=$h timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --steps 20 --warmup 6 > gpurun_out/prof11/$name.log 2>&1 || { echo "prof $name failed"; tail -30 gpurun_out/prof11/$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/p_$name gpurun_out/prof11/${name}_summary.txt --steps 20 > /dev/null || exit 1
  rm -rf /tmp/p_$name
  head -1 gpurun_out/prof11/${name}_summary.txt
done
