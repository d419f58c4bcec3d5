# LeNet with a 2048-key candidate floor for few-k tensors: misses per tensor, EF and no-EF times
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py tests/e2e/test_gpu_train.py" TESTS_K="topk or one_launch or predict or lenet" bash tools/gpurun_suite.sh tests && \
for a in "--preset lenet --no-extras --error-feedback off" "--preset lenet --no-extras"; do
  timeout -k 10 300 python bench.py $a --steps 200 --warmup 20 > /tmp/b.txt 2>/dev/null || exit 1
  grep '^{' /tmp/b.txt | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("codec_health"))'
done && \
bash tools/gpurun_suite.sh ab 3 "noef||--preset lenet --no-extras --error-feedback off" "ef||--preset lenet --no-extras"
