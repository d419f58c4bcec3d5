# Segmented-graph overlap A/B (world of one with a real RCCL communicator: EWDML_FORCE_PG=1)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
PORT=29611
B() {  # name, bench args
  name=$1; shift
  PORT=$((PORT+1))
  out=$(EWDML_FORCE_PG=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
      --master-addr 127.0.0.1 --master-port $PORT bench.py --gpus 1 --steps 40 --warmup 6 --no-extras "$@" \
      2>>gpurun_out/overlap_err.log | grep '^{') || { echo "FAILED $name"; tail -20 gpurun_out/overlap_err.log; exit 1; }
  echo "$out" >> gpurun_out/overlap.jsonl
  echo "$name $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["host_enqueue_ms_per_step"], d["config"]["hip_graph"], d["config"]["buckets"], d["config"]["comm"], d.get("overlap_effective"), d.get("overlap_comm_graphs"))')"
}
for r in 1; do
B vgg_dense_full_b64 --compress none --hip-graph full
B vgg_dense_full_b8 --compress none --hip-graph full --bucket-mb 8
B vgg_dense_seg_b8 --compress none --hip-graph segmented --bucket-mb 8
B vgg_dense_seg1_b4 --compress none --hip-graph segmented --bucket-mb 4 --extra "--overlap-splits 1"
B vgg_topk_full_b64 --hip-graph full
B vgg_topk_seg1_b4 --hip-graph segmented --bucket-mb 4
B r50_dense_full --preset resnet50_cifar --compress none --hip-graph full
B r50_dense_seg_b16 --preset resnet50_cifar --compress none --hip-graph segmented --bucket-mb 16
B r50_dense_seg1_b8 --preset resnet50_cifar --compress none --hip-graph segmented --bucket-mb 8
done
# kernel trace of the segmented dense VGG step (world of one, real RCCL communicator)
export EWDML_FORCE_PG=1 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0 MASTER_ADDR=127.0.0.1 MASTER_PORT=29688 EWDML_PROF_GAP=1
rm -rf /tmp/p_seg
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_seg -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 6 --no-extras --compress none --hip-graph segmented --bucket-mb 4 > gpurun_out/prof_seg.log 2>&1 || { tail -20 gpurun_out/prof_seg.log; exit 1; }
python3 tools/overlap_check.py /tmp/p_seg --steps 20 --out gpurun_out/overlap_vgg_dense_seg.txt | head -20
python3 tools/prof_summarize.py /tmp/p_seg gpurun_out/prof_vgg_dense_seg.txt --steps 20 > /dev/null
rm -rf /tmp/p_seg
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_seg -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 6 --no-extras --hip-graph segmented --bucket-mb 4 > gpurun_out/prof_seg2.log 2>&1 || { tail -20 gpurun_out/prof_seg2.log; exit 1; }
python3 tools/overlap_check.py /tmp/p_seg --steps 20 --out gpurun_out/overlap_vgg_topk_seg.txt | head -20
