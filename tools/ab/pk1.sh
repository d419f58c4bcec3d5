set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" bash tools/gpurun_suite.sh tests && \
EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py && \
bash tools/gpurun_suite.sh bench "--preset lenet --no-extras" "--preset lenet --no-extras --error-feedback off" "--preset lenet --no-extras --compress none"
