# decode A/B: this tree's build vs tools/alt/_C_head.so at N = 1..8 ranks' payloads
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 300 $T tests/kernels/test_hip_codecs.py -k decode > gpurun_out/dec_tests.log 2>&1 || { tail -40 gpurun_out/dec_tests.log; exit 1; }
tail -1 gpurun_out/dec_tests.log
for i in 1 2; do
  echo "== new"; timeout -k 10 120 python -u tools/probes/decode_probe.py || exit 1
  echo "== head"; EWDML_EXT=tools/alt/_C_head.so timeout -k 10 120 python -u tools/probes/decode_probe.py || exit 1
done
