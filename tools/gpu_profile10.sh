#!/bin/bash
# kernel profiles of the current defaults: VGG-11 (top-k+QSGD), VGG-11 dense, ResNet-50 CIFAR
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/prof10
export TMPDIR=/tmp EWDML_PROF_GAP=1
for v in "vgg11_topk:" "vgg11_dense:--compress none" "r50c_topk:--preset resnet50_cifar"; do
  name=${v%%:*}; args=${v#*:}
  timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_$name -o run -- python3 bench.py --steps 20 --warmup 6 $args > gpurun_out/prof10/$name.log 2>&1 || { echo "prof $name failed"; tail -30 gpurun_out/prof10/$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/p_$name gpurun_out/prof10/${name}_summary.txt --steps 20 > /dev/null || exit 1
  rm -rf /tmp/p_$name
  head -1 gpurun_out/prof10/${name}_summary.txt
done
