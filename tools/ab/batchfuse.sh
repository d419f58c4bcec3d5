# LeNet batch formed in the conv launch (EWDML_BATCH_IN_MODEL): LeNet / loader / accuracy tests, A/B
set -o pipefail
TESTS_ARGS="tests/e2e tests/kernels/test_lenet_fused.py tests/unit" TESTS_K="lenet or loader or batch or mnist" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "fused||--preset lenet --no-extras" "sep|EWDML_BATCH_IN_MODEL=0|--preset lenet --no-extras"
