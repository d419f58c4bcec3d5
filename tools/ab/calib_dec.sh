set -o pipefail
mkdir -p gpurun_out/calib
timeout -k 10 120 python tools/probes/decode_probe.py --model ResNet50 --json gpurun_out/calib/decode_resnet50.json && \
timeout -k 10 120 python tools/probes/decode_probe.py --model LeNet --json gpurun_out/calib/decode_lenet.json && \
timeout -k 10 120 python tools/probes/decode_probe.py --model resnet50_imagenet --ratio 0.001 --bits 4 --json gpurun_out/calib/decode_resnet50_imagenet.json
