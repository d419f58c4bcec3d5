set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="dense_apply" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "noef_apply||--preset lenet --no-extras --error-feedback off" "noef_decode|EWDML_LOCAL_APPLY=0|--preset lenet --no-extras --error-feedback off" "ef||--preset lenet --no-extras"
