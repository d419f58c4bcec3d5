set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp EWDML_ORACLE=1 EWDML_GRAD_VIEWS=1
mkdir -p gpurun_out
P="python -u tools/ef_probe.py --device cuda --batch 128 --steps 300 --synthetic 16384 --hip-graph off"
LW="--lr-warmup-epochs 1 --lr-warmup-start 0.1"
run() { timeout -k 10 400 $P "$@" >> gpurun_out/ef_sweep3.jsonl 2>> gpurun_out/ef_sweep.err || { tail -20 gpurun_out/ef_sweep.err; exit 1; }; tail -1 gpurun_out/ef_sweep3.jsonl | cut -c1-150; }
run --modes ef21,local --extra "$LW"
run --modes ef21,local --warmup 0.25,0.0625,0.015625 --extra "$LW"
run --modes ef21,dgc
