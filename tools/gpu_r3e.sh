set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -v --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/e2e/test_gpu_train.py -k "ps_worker" > gpurun_out/ps_graph.log 2>&1 || { tail -60 gpurun_out/ps_graph.log; exit 1; }
tail -3 gpurun_out/ps_graph.log
timeout -k 10 900 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/gpu_all.log 2>&1 || { grep -E "FAIL|Error|passed|failed" gpurun_out/gpu_all.log | tail -40; exit 1; }
tail -3 gpurun_out/gpu_all.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { tail -30 gpurun_out/smoke.log; exit 1; }
tail -2 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
