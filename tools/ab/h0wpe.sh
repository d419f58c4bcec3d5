set -o pipefail
bash tools/gpurun_suite.sh ab 3 "base||--no-extras" "w5|EWDML_PK_H0_WPE=5|--no-extras" "w4|EWDML_PK_H0_WPE=4|--no-extras" && \
EWDML_PK1_STAMPS=1 timeout -k 10 120 python tools/probes/pk1_stamps.py
