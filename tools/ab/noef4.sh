# LeNet without error feedback: miss types per tensor
set -o pipefail
timeout -k 10 300 python bench.py --preset lenet --no-extras --error-feedback off --steps 200 --warmup 20 > /tmp/b.txt 2>/dev/null && \
grep '^{' /tmp/b.txt | tail -1 | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d.get("codec_health"))'
