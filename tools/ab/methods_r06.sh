# time to accuracy per method on the MI355X at the round-6 kernels
set -o pipefail
PY_TIMEOUT=900 bash tools/gpurun_suite.sh py tools/methods_eval.py --device cuda --steps 1500 --ratio 0.4 \
  --targets 97,98 --json gpurun_out/methods_eval_gpu_r06.json --out-gpu gpurun_out/methods_gpu_r06.md > gpurun_out/methods_r06.log 2>&1
rc=$?; tail -5 gpurun_out/methods_r06.log; exit $rc
