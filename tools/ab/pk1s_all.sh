# k_pk_one stamps with every <= 8192-element tensor keeping all its elements as candidates
set -o pipefail
EWDML_CAND_ALL_MAX=8192 EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py > gpurun_out/pk1s_all.txt 2>&1 && cat gpurun_out/pk1s_all.txt
