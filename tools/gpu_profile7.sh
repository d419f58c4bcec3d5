#!/bin/bash
# kernel profile of the fused NHWC default (topk+qsgd and dense), then batch-size sweep
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof7
export TMPDIR=/tmp EWDML_PROF_GAP=1
for v in "topk_fused:" "dense_fused:--compress none"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --steps 20 --warmup 6 $args > gpurun_out/prof7/$name.log 2>&1 || { echo "prof $name failed"; tail -30 gpurun_out/prof7/$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/p_$name gpurun_out/prof7/${name}_summary.txt --steps 20 > /dev/null || exit 1
  rm -rf /tmp/p_$name
done
unset EWDML_PROF_GAP
rm -f gpurun_out/ab.log
bash tools/ab.sh 2 "b128|EWDML_X=0|" "b128_dense|EWDML_X=0|--compress none"
