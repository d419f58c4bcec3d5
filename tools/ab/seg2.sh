set -o pipefail
export EWDML_FORCE_PG=1
TESTS_ARGS="tests/e2e/test_gpu_train.py tests/kernels/test_hip_codecs.py" TESTS_K="segmented or one_launch or apply or predictive" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 2 "full16||--compress none --no-extras --hip-graph full" "full1||--compress none --no-extras --hip-graph full --graph-unroll 1" "seg_dev||--compress none --no-extras --hip-graph segmented" "seg_evt|EWDML_SEG_HANDOFF=event|--compress none --no-extras --hip-graph segmented" "seg_dev_b8||--compress none --no-extras --hip-graph segmented --bucket-mb 8" "seg_evt_b8|EWDML_SEG_HANDOFF=event|--compress none --no-extras --hip-graph segmented --bucket-mb 8" && \
unset EWDML_FORCE_PG && bash tools/gpurun_suite.sh bench "--preset lenet --no-extras" "--preset lenet --no-extras --error-feedback off"
