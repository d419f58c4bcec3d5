#!/bin/bash
# A/B: HIP_FORCE_DEV_KERNARG=1 (package default) vs 0, all presets, unprofiled
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/karg
for p in vgg11 vgg11 lenet resnet50_cifar resnet50_imagenet; do
  for v in 1 0; do
    HIP_FORCE_DEV_KERNARG=$v timeout -k 10 300 python bench.py --preset $p > gpurun_out/karg/$p.$v.json 2> gpurun_out/karg/err.log || { tail -20 gpurun_out/karg/err.log; exit 1; }
    python3 -c "import json,sys; r=json.loads(open('gpurun_out/karg/$p.$v.json').read().strip().splitlines()[-1]); print('$p', 'kernarg_dev=$v', r['value'], r['ms_per_step'])"
  done
done
