# ranked bin with wave-aggregated compaction / vector rank loop: tests, stamps, LeNet A/B
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="one_launch or predict" bash tools/gpurun_suite.sh tests && \
EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py > gpurun_out/pk1s.txt 2>&1 && grep -E "tensor 4|span|stats" gpurun_out/pk1s.txt && \
bash tools/gpurun_suite.sh ab 3 "lenet||--preset lenet --no-extras" "lenet_norank|EWDML_PK_RANK=0|--preset lenet --no-extras"
