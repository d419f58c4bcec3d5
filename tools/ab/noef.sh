# LeNet without error feedback (Method 5 as published): encode fast / full counts and a trace
set -o pipefail
for a in "--preset lenet --no-extras" "--preset lenet --no-extras --error-feedback off"; do
  timeout -k 10 300 python bench.py $a --steps 200 --warmup 20 > /tmp/b.txt 2>/dev/null || exit 1
  grep '^{' /tmp/b.txt | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("codec_health"))'
done
bash tools/gpurun_suite.sh prof lenet_noef "--preset lenet --steps 40 --error-feedback off" > /dev/null && head -12 gpurun_out/prof_lenet_noef.txt
