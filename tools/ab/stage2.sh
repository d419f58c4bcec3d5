set -o pipefail
TESTS_ARGS="tests/e2e/test_gpu_train.py" TESTS_K="producer_staging" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "stage||--no-extras" "nostage|EWDML_PRODUCER_STAGE=0|--no-extras" && \
bash tools/gpurun_suite.sh prof vgg_stage "--steps 20" && EWDML_PRODUCER_STAGE=0 bash tools/gpurun_suite.sh prof vgg_nostage "--steps 20"
