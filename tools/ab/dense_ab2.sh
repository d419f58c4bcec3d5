set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh ab 3 "noef||--preset lenet --no-extras --error-feedback off" "ef||--preset lenet --no-extras" "vgg||--no-extras" && \
bash tools/gpurun_suite.sh bench "--preset lenet --no-extras --error-feedback off" && tail -1 gpurun_out/bench.jsonl | python3 -c "import sys,json; print(json.loads(sys.stdin.read())['codec_health'])"
