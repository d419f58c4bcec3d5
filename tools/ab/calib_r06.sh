# Round-6 N = 1 measurements for the step model (tools/step_model_calibrate.py): preset lines,
# the N > 1 code path at world 1 (EWDML_LOCAL_APPLY=0), segmented vs one-graph steps with the real
# communicator, and the decode at 1/2/4/8 payloads.
set -o pipefail
rm -f gpurun_out/bench.jsonl gpurun_out/ab.log
mkdir -p gpurun_out/calib
bash tools/gpurun_suite.sh bench "--no-extras" "--no-extras --compress none" \
  "--preset lenet --no-extras" "--preset lenet --no-extras --compress none" \
  "--preset resnet50_cifar --no-extras" "--preset resnet50_cifar --no-extras --compress none" \
  "--preset resnet50_imagenet --no-extras" "--preset resnet50_imagenet --no-extras --compress none" && \
cp gpurun_out/bench.jsonl gpurun_out/calib/presets.jsonl && rm gpurun_out/bench.jsonl && \
EWDML_LOCAL_APPLY=0 bash tools/gpurun_suite.sh bench "--no-extras" "--preset lenet --no-extras" \
  "--preset resnet50_cifar --no-extras" "--preset resnet50_imagenet --no-extras" && \
cp gpurun_out/bench.jsonl gpurun_out/calib/no_local_apply.jsonl && rm gpurun_out/bench.jsonl && \
EWDML_FORCE_PG=1 bash tools/gpurun_suite.sh bench "--no-extras --compress none --hip-graph full --graph-unroll 1" \
  "--no-extras --compress none --hip-graph segmented" \
  "--preset resnet50_cifar --no-extras --compress none --hip-graph full --graph-unroll 1" \
  "--preset resnet50_cifar --no-extras --compress none --hip-graph segmented" \
  "--no-extras --hip-graph full --graph-unroll 1" \
  "--no-extras --hip-graph segmented" && \
cp gpurun_out/bench.jsonl gpurun_out/calib/segmented.jsonl && rm gpurun_out/bench.jsonl && \
timeout -k 10 120 python tools/probes/decode_probe.py --model VGG11 --json gpurun_out/calib/decode_vgg11.json && \
timeout -k 10 120 python tools/probes/decode_probe.py --model ResNet50 --json gpurun_out/calib/decode_resnet50.json && \
timeout -k 10 120 python tools/probes/decode_probe.py --model LeNet --json gpurun_out/calib/decode_lenet.json && \
timeout -k 10 120 python tools/probes/decode_probe.py --model resnet50_imagenet --ratio 0.001 --bits 4 --json gpurun_out/calib/decode_resnet50_imagenet.json
