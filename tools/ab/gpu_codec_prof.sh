# codec bit-exactness + Method 6 RCCL capture + headline profile (no extras)
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 400 $T tests/kernels/test_hip_codecs.py > gpurun_out/codec_tests.log 2>&1 || { tail -40 gpurun_out/codec_tests.log; exit 1; }
tail -1 gpurun_out/codec_tests.log
timeout -k 10 400 $T tests/e2e/test_gpu_train.py -k "method6 or rccl or ef" > gpurun_out/m6_tests.log 2>&1 || { tail -40 gpurun_out/m6_tests.log; exit 1; }
tail -1 gpurun_out/m6_tests.log
bash tools/gpurun_suite.sh prof vgg11_fp32 "--no-extras"
