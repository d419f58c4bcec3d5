set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_hip_codecs.py tests/e2e/test_watchdog.py -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_tests.log 2>&1 || { tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
timeout -k 10 600 python -u -m pytest tests/kernels/test_conv_f32.py -x -q --timeout 120 --timeout-method thread -k "deferred or autograd_grad" > gpurun_out/conv_tests.log 2>&1 || { tail -40 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
P="python -u tools/ef_probe.py --device cuda --batch 128 --steps 300 --synthetic 16384 --hip-graph full"
run() { timeout -k 10 300 $P "$@" >> gpurun_out/ef_sweep.jsonl 2>> gpurun_out/ef_sweep.err || { tail -20 gpurun_out/ef_sweep.err; exit 1; }; tail -1 gpurun_out/ef_sweep.jsonl | cut -c1-220; }
run --compress none --modes none
run --modes none,plain,dgc
run --modes dgc --warmup 0.25,0.0625,0.015625
run --modes dgc --warmup 0.25,0.0625,0.015625 --dense-below 4096
run --modes plain --warmup 0.25,0.0625,0.015625 --dense-below 4096
