# Round-6 traces: LeNet (one-launch codec + local apply), ResNet-50 224 px (non-native kernels),
# VGG-11 per-kernel roofline (trace + two PMC passes).
set -o pipefail
bash tools/gpurun_suite.sh prof lenet_r06 "--preset lenet --steps 40" && \
bash tools/gpurun_suite.sh prof r50i_r06 "--preset resnet50_imagenet --steps 10" && \
bash tools/ab/gpu_roofline.sh vgg11_r06 ""
