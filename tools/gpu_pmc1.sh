#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --output-format csv -d /tmp/pmc1 -- python3 tools/conv_pmc.py > gpurun_out/pmc/run1.log 2>&1 || { tail -20 gpurun_out/pmc/run1.log; exit 1; }
python3 tools/pmc_summarize.py /tmp/pmc1 k_ > gpurun_out/pmc/pass1.txt; cat gpurun_out/pmc/pass1.txt
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d /tmp/pmc2 -- python3 tools/conv_pmc.py > gpurun_out/pmc/run2.log 2>&1 || { tail -20 gpurun_out/pmc/run2.log; exit 1; }
python3 tools/pmc_summarize.py /tmp/pmc2 k_ > gpurun_out/pmc/pass2.txt; cat gpurun_out/pmc/pass2.txt
