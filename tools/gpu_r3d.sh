set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/kernels/test_hip_codecs.py -k "dgc or decode or encode" > gpurun_out/codec_tests.log 2>&1 || { tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
P="python -u tools/ef_probe.py --device cuda --batch 128 --steps 400 --synthetic 16384 --hip-graph full"
LW="--lr-warmup-epochs 1 --lr-warmup-start 0.1"
LW2="--lr-warmup-epochs 2 --lr-warmup-start 0.1"
W3="0.25,0.0625,0.015625"
W5="0.25,0.125,0.0625,0.03125,0.015625"
run() { timeout -k 10 300 $P "$@" >> gpurun_out/ef_sweep4.jsonl 2>> gpurun_out/ef_sweep.err || { tail -20 gpurun_out/ef_sweep.err; exit 1; }; tail -1 gpurun_out/ef_sweep4.jsonl | cut -c1-120; }
run --compress none --modes none --extra "$LW"
run --compress none --modes none --extra "$LW2"
run --modes local,dgc --warmup $W3 --extra "$LW"
run --modes local,dgc --warmup $W5 --warmup-epochs 2 --extra "$LW2"
run --modes local --warmup $W5 --warmup-epochs 2 --extra "$LW"
run --modes none --extra "$LW2"
