#!/bin/bash
# Kernel trace + two --pmc passes of one bench.py configuration, joined into a per-kernel roofline
# table (tools/roofline.py).  gpurun --timeout 900 -- bash tools/ab/gpu_roofline.sh NAME "ARGS"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
name=${1:-vgg11}; args=${2:-}
steps=20
rm -rf /tmp/rf_${name}_*
EWDML_PROF_GAP=1 timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d /tmp/rf_${name}_trace \
    -o run -- python3 bench.py $args --no-extras --steps $steps --warmup 6 > gpurun_out/rf_${name}_trace.log 2>&1 \
    || { echo "trace failed"; tail -30 gpurun_out/rf_${name}_trace.log; exit 1; }
python3 tools/prof_summarize.py /tmp/rf_${name}_trace gpurun_out/rf_${name}_graph.txt --steps $steps > /dev/null || exit 1
grep '^{' gpurun_out/rf_${name}_trace.log | tail -1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
    --kernel-trace --output-format csv -d /tmp/rf_${name}_a -o run -- python3 bench.py $args --no-extras \
    --steps 5 --warmup 4 > gpurun_out/rf_${name}_a.log 2>&1 || { echo "pmc a failed"; tail -30 gpurun_out/rf_${name}_a.log; exit 1; }
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAVES \
    --kernel-trace --output-format csv -d /tmp/rf_${name}_b -o run -- python3 bench.py $args --no-extras \
    --steps 5 --warmup 4 > gpurun_out/rf_${name}_b.log 2>&1 || { echo "pmc b failed"; tail -30 gpurun_out/rf_${name}_b.log; exit 1; }
python3 tools/roofline.py /tmp/rf_${name}_trace gpurun_out/roofline_${name}.txt --steps $steps \
    /tmp/rf_${name}_a /tmp/rf_${name}_b || exit 1
python3 tools/pmc_summarize.py /tmp/rf_${name}_a > gpurun_out/rf_${name}_pmc_a.txt
python3 tools/pmc_summarize.py /tmp/rf_${name}_b > gpurun_out/rf_${name}_pmc_b.txt
