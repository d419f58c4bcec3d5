# codec / decode / local SGD GPU checks after the sparse decode and Method 6 graph changes
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/kernels/test_hip_codecs.py > gpurun_out/codec_tests.log 2>&1 || { tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
timeout -k 10 400 $T tests/e2e/test_gpu_train.py -k "method6 or local_sgd" > gpurun_out/m6_tests.log 2>&1 || { tail -40 gpurun_out/m6_tests.log; exit 1; }
tail -1 gpurun_out/m6_tests.log
timeout -k 10 400 python -u bench.py > gpurun_out/bench_default.log 2>&1 || { tail -30 gpurun_out/bench_default.log; exit 1; }
tail -1 gpurun_out/bench_default.log
