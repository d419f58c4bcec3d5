set -o pipefail
cd $GRAFT_REPO_ROOT
P="timeout -k 10 120 python -u tools/conv_f32_probe.py"
timeout -k 10 300 python -u -m pytest tests/kernels/test_conv_f32.py -x -q --timeout 200 --timeout-method thread > gpurun_out/t_f32.log 2>&1; tail -2 gpurun_out/t_f32.log
$P && EWDML_CF_PLAN=128,128,1 $P --shapes big --dirs fwd,bwd
