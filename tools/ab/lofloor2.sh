# floor without EF only: codec tests, LeNet EF / no-EF at the default steps
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" TESTS_K="topk or one_launch or predict or lenet" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "ef||--preset lenet --no-extras" "noef||--preset lenet --no-extras --error-feedback off"
