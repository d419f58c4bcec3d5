# candidate write: one load per candidate, the first prefetched during the wait: tests, stamps, A/B
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" TESTS_K="topk or one_launch or predict or lenet or apply" bash tools/gpurun_suite.sh tests && \
EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py > gpurun_out/pk1s.txt 2>&1 && grep -E "tensor 4|span" gpurun_out/pk1s.txt && \
bash tools/gpurun_suite.sh ab 3 "lenet||--preset lenet --no-extras" "vgg||--no-extras"
