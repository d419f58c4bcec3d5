mkdir -p gpurun_out
bash tools/gpurun_suite.sh prof pk_vgg "--no-extras --steps 20" > gpurun_out/combo_prof.txt 2>&1 || { tail -20 gpurun_out/combo_prof.txt; exit 1; }
head -3 gpurun_out/prof_pk_vgg.txt; grep -E "k_pk|k_topk" gpurun_out/prof_pk_vgg.txt | head -8
timeout -k 10 300 python tools/probes/decode_probe.py > gpurun_out/decode_probe.txt 2>&1 || { tail gpurun_out/decode_probe.txt; exit 1; }
cat gpurun_out/decode_probe.txt
bash tools/probes/gpu_graph_shape.sh || exit 1
