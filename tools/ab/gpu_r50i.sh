# ResNet-50 224px fp32: native stride-2 convs vs MIOpen A/B, then a kernel profile
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpurun_suite.sh ab 2 "s2native|EWDML_CONV_S2=1|--preset resnet50_imagenet --no-extras" "s2miopen|EWDML_CONV_S2=0|--preset resnet50_imagenet --no-extras" || exit 1
bash tools/gpurun_suite.sh prof r50i "--preset resnet50_imagenet --no-extras --steps 10 --warmup 6"
