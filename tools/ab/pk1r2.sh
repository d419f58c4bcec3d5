# ranked digit-0 bin, A/B against the radix digits 1 and 2 (EWDML_PK_RANK=0, no compaction)
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="one_launch or predict" bash tools/gpurun_suite.sh tests && \
EWDML_PK_RANK=0 TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="one_launch or predict" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "lenet||--preset lenet --no-extras" "lenet_norank|EWDML_PK_RANK=0|--preset lenet --no-extras" \
  "lenet_noef||--preset lenet --no-extras --error-feedback off" "lenet_noef_norank|EWDML_PK_RANK=0|--preset lenet --no-extras --error-feedback off"
