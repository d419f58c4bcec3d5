set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh bench "--preset lenet --no-extras" "--preset lenet --no-extras --error-feedback off" "--no-extras" && \
bash tools/gpurun_suite.sh prof lenet_one "--preset lenet --steps 40"
