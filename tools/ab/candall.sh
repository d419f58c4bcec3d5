# small tensors keep all elements as candidates (EWDML_CAND_ALL_MAX) with the register write for
# candidate-heavy chunks: codec tests (both settings), stamps, A/B
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" TESTS_K="topk or one_launch or predict or lenet" bash tools/gpurun_suite.sh tests && \
EWDML_CAND_ALL_MAX=8192 TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="topk or one_launch or predict" bash tools/gpurun_suite.sh tests && \
EWDML_CAND_ALL_MAX=8192 EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py > gpurun_out/pk1s_all.txt 2>&1 && grep -E "tensor|span" gpurun_out/pk1s_all.txt && \
bash tools/gpurun_suite.sh ab 3 "noef_all|EWDML_CAND_ALL_MAX=8192|--preset lenet --no-extras --error-feedback off" "noef||--preset lenet --no-extras --error-feedback off" \
  "ef_all|EWDML_CAND_ALL_MAX=8192|--preset lenet --no-extras" "ef||--preset lenet --no-extras" "vgg_all|EWDML_CAND_ALL_MAX=8192|--no-extras" "vgg||--no-extras"
