mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/kernels/test_hip_codecs.py -x -q --timeout 120 --timeout-method thread > gpurun_out/codec_tests.log 2>&1; rc=$?; tail -3 gpurun_out/codec_tests.log; [ $rc -eq 0 ] || exit 1
bash tools/gpurun_suite.sh prof pk_vgg "--no-extras --steps 20" > gpurun_out/combo_prof.txt 2>&1 || { tail -20 gpurun_out/combo_prof.txt; exit 1; }
head -3 gpurun_out/prof_pk_vgg.txt; grep -E "k_pk|k_topk" gpurun_out/prof_pk_vgg.txt | head -8
timeout -k 10 300 python tools/probes/decode_probe.py > gpurun_out/decode_probe.txt 2>&1 || { tail gpurun_out/decode_probe.txt; exit 1; }
cat gpurun_out/decode_probe.txt
bash tools/probes/gpu_graph_shape.sh || exit 1
