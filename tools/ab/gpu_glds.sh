# LDS-DMA forward GEMM: bitwise test vs the register-staged kernel, then per-layer timing A/B
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/kernels/test_conv_f32.py -k "lds_dma or forward" > gpurun_out/glds_tests.log 2>&1 || { tail -40 gpurun_out/glds_tests.log; exit 1; }
tail -2 gpurun_out/glds_tests.log
for g in 0 1 0 1; do
  echo "== GLDS=$g"
  EWDML_CF_GLDS=$g timeout -k 10 120 python -u tools/probes/conv_f32_probe.py --dirs fwd --wino > gpurun_out/glds_probe_$g.txt 2>&1 || { tail -20 gpurun_out/glds_probe_$g.txt; exit 1; }
  grep -i "total\|TF" gpurun_out/glds_probe_$g.txt | tail -14
  EWDML_CF_GLDS=$g timeout -k 10 120 python -u tools/probes/conv_f32_probe.py --dirs fwd --shapes big 2>&1 | tail -3
done
