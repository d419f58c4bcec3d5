set -o pipefail
export EWDML_FORCE_PG=1
TESTS_K="deferred_reduction or flat_view or deferred_transform or unrolled" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 2 "full16||--compress none --no-extras --hip-graph full" "full1||--compress none --no-extras --hip-graph full --graph-unroll 1" "seg||--compress none --no-extras --hip-graph segmented" "seg_b64||--compress none --no-extras --hip-graph segmented --bucket-mb 64" && \
bash tools/gpurun_suite.sh prof segdense "--compress none --hip-graph segmented --steps 20" && \
bash tools/gpurun_suite.sh prof full1dense "--compress none --hip-graph full --graph-unroll 1 --steps 20"
