# final round-6 step traces: VGG-11 (headline) and LeNet
set -o pipefail
bash tools/gpurun_suite.sh prof vgg_final "--steps 20" > /dev/null && \
bash tools/gpurun_suite.sh prof lenet_final "--preset lenet --steps 40" > /dev/null && \
head -3 gpurun_out/prof_vgg_final.txt && head -10 gpurun_out/prof_lenet_final.txt
