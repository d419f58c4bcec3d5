# after the prefetch bound fix: the codec tests in full, then the one-launch / trainer subset
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="" bash tools/gpurun_suite.sh tests && \
TESTS_ARGS="tests/e2e/test_gpu_train.py" TESTS_K="topk or lenet or apply or one_launch" bash tools/gpurun_suite.sh tests
