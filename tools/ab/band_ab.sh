set -o pipefail
bash tools/gpurun_suite.sh ab 3 "base||--no-extras" "b6_10|EWDML_PK_BAND=6,10|--no-extras" "b5_8|EWDML_PK_BAND=5,8|--no-extras" "b6_12_w4|EWDML_PK_BAND=6,12 EWDML_PK_H0_WPE=4|--no-extras" "w4|EWDML_PK_H0_WPE=4|--no-extras"
