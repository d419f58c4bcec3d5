set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/e2e/test_gpu_train.py -k "local_sgd or graph_modes" > gpurun_out/lsgd_tests.log 2>&1 || { tail -60 gpurun_out/lsgd_tests.log; exit 1; }
tail -12 gpurun_out/lsgd_tests.log
timeout -k 10 400 python -u bench.py --steps 40 --warmup 8 --no-extras --error-feedback off --extra "--method 6" > gpurun_out/m6.log 2>&1 || { tail -30 gpurun_out/m6.log; exit 1; }
tail -1 gpurun_out/m6.log | cut -c1-300
