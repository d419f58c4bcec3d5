# LeNet / VGG-11 without error feedback: which tensors miss the predicted bound
set -o pipefail
TESTS_ARGS="tests/kernels/test_hip_codecs.py" TESTS_K="predict or one_launch or stats or lookback" bash tools/gpurun_suite.sh tests && \
for a in "--preset lenet --no-extras --error-feedback off" "--preset lenet --no-extras" "--no-extras --error-feedback off"; do
  timeout -k 10 300 python bench.py $a --steps 200 --warmup 20 > /tmp/b.txt 2>/dev/null || exit 1
  grep '^{' /tmp/b.txt | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("codec_health"))'
done
