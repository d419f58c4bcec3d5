set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py tests/kernels/test_conv_f32.py" TESTS_K="apply or one_launch or fenced or winograd or vgg11" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh bench "--preset lenet --no-extras" "--preset lenet --no-extras --error-feedback off" "--no-extras"
