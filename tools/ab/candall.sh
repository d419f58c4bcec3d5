# small tensors keep all elements as candidates (compress/plan.py CAND_ALL_MAX): codec tests, A/B
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" TESTS_K="topk or one_launch or predict or lenet" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "noef||--preset lenet --no-extras --error-feedback off" "noef_old|EWDML_CAND_ALL_MAX=0|--preset lenet --no-extras --error-feedback off" \
  "ef||--preset lenet --no-extras" "ef_old|EWDML_CAND_ALL_MAX=0|--preset lenet --no-extras" "vgg||--no-extras" "vgg_old|EWDML_CAND_ALL_MAX=0|--no-extras"
