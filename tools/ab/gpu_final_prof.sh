# end-of-round profiles of the headline and the ResNet-50 presets at HEAD
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpurun_suite.sh prof vgg11_fp32 "--no-extras" > /dev/null || exit 1
bash tools/gpurun_suite.sh prof r50c "--preset resnet50_cifar --no-extras --steps 10 --warmup 6" > /dev/null || exit 1
bash tools/gpurun_suite.sh prof r50i "--preset resnet50_imagenet --no-extras --steps 10 --warmup 6" > /dev/null || exit 1
for f in vgg11_fp32 r50c r50i; do head -1 gpurun_out/prof_$f.txt; done
