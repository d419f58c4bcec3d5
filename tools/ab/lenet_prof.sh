set -o pipefail
bash tools/gpurun_suite.sh prof lenet_ef "--preset lenet --steps 40" && \
bash tools/gpurun_suite.sh prof lenet_noef "--preset lenet --steps 40 --error-feedback off" && \
bash tools/gpurun_suite.sh prof lenet_dense "--preset lenet --steps 40 --compress none"
