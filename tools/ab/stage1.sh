set -o pipefail
TESTS_ARGS="tests/e2e/test_gpu_train.py tests/kernels/test_hip_codecs.py tests/kernels/test_conv_f32.py" TESTS_K="producer_staging or smallmap or one_launch or apply or predictive" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "stage||--no-extras" "nostage|EWDML_PRODUCER_STAGE=0|--no-extras"
