set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh bench "--preset lenet --no-extras" "--preset lenet --no-extras --error-feedback off" "--no-extras" "--no-extras --compress none"
