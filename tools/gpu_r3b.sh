set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/kernels/test_hip_codecs.py tests/e2e/test_watchdog.py > gpurun_out/codec_tests.log 2>&1 || { tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
timeout -k 10 600 $T tests/e2e/test_gpu_train.py > gpurun_out/train_tests.log 2>&1 || { tail -40 gpurun_out/train_tests.log; exit 1; }
tail -1 gpurun_out/train_tests.log
P="python -u tools/ef_probe.py --device cuda --batch 128 --steps 300 --synthetic 16384 --hip-graph full"
LW="--lr-warmup-epochs 1 --lr-warmup-start 0.1"
run() { timeout -k 10 300 $P "$@" >> gpurun_out/ef_sweep2.jsonl 2>> gpurun_out/ef_sweep.err || { tail -20 gpurun_out/ef_sweep.err; exit 1; }; tail -1 gpurun_out/ef_sweep2.jsonl | cut -c1-200; }
run --compress none --modes none --extra "$LW"
run --modes none,dgc --extra "$LW"
run --modes dgc --warmup 0.25,0.0625,0.015625 --extra "$LW"
run --modes dgc --warmup 0.25,0.0625,0.015625 --dense-below 4096 --extra "$LW"
