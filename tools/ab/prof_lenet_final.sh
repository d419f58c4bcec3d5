set -o pipefail
bash tools/gpurun_suite.sh prof lenet_final "--preset lenet --steps 40" > /dev/null && head -10 gpurun_out/prof_lenet_final.txt
