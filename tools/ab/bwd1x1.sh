set -o pipefail
timeout -k 10 180 python tools/probes/bwd1x1_probe.py > gpurun_out/bwd1x1.txt 2>&1; cat gpurun_out/bwd1x1.txt
