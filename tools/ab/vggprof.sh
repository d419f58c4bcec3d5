set -o pipefail
bash tools/gpurun_suite.sh prof vgg_apply "--steps 20" && \
EWDML_LOCAL_APPLY=0 bash tools/gpurun_suite.sh prof vgg_noapply "--steps 20"
