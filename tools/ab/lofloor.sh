# candidate band floor for few-k tensors (EWDML_PK1_LO) at the bench's default steps, EF and no-EF
set -o pipefail
for r in 1 2 3; do
  for v in "lo2048|EWDML_PK1_LO=2048|--preset lenet --no-extras" "lo0|EWDML_PK1_LO=0|--preset lenet --no-extras" \
           "noef_lo2048|EWDML_PK1_LO=2048|--preset lenet --no-extras --error-feedback off" "noef_lo0|EWDML_PK1_LO=0|--preset lenet --no-extras --error-feedback off"; do
    IFS='|' read -r name envs args <<< "$v"
    out=$(env $envs timeout -k 10 300 python bench.py $args 2>/dev/null | grep '^{') || exit 1
    echo "$name r$r $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["codec_health"]["topk_encode_full"])')" | tee -a gpurun_out/ab.log
  done
done
