# k_pk_one phase stamps incl. the select's sub-phases (LeNet bucket)
set -o pipefail
EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py > gpurun_out/pk1s.txt 2>&1 && cat gpurun_out/pk1s.txt
