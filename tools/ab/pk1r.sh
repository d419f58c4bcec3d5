# ranked digit-0 bin in both selects (one-launch and three-launch): codec tests, stamps, A/B
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" TESTS_K="one_launch or topk or lenet or apply or predict" bash tools/gpurun_suite.sh tests && \
EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py > gpurun_out/pk1s.txt 2>&1 && grep -E "tensor 4|span|stats" gpurun_out/pk1s.txt && \
bash tools/gpurun_suite.sh ab 3 "lenet||--preset lenet --no-extras" "lenet_norank|EWDML_PK_RANK=0|--preset lenet --no-extras" \
  "vgg||--no-extras" "vgg_norank|EWDML_PK_RANK=0|--no-extras"
