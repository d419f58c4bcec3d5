set -o pipefail
TESTS_ARGS="tests/e2e/test_gpu_accuracy.py" TESTS_K="lenet" bash tools/gpurun_suite.sh tests && \
bash tools/gpurun_suite.sh bench "--preset lenet" && tail -1 gpurun_out/bench.jsonl | python3 -c "import sys,json; d=json.loads(sys.stdin.read()); print({k:v for k,v in d.items() if k.startswith(('value','ms_per','dtype','model_err','predicted'))})"
