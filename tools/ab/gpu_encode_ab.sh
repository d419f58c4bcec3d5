# encode A/B: per-kernel times of the top-k encode for this tree's build and tools/alt/_C_*.so
set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp; mkdir -p gpurun_out
for v in cur $(ls tools/alt | sed -n 's/^_C_\(.*\)\.so$/\1/p'); do
  ext=""; [ "$v" != cur ] && ext=tools/alt/_C_$v.so
  rm -rf /tmp/pe_$v
  EWDML_EXT=$ext timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pe_$v -o run -- python3 tools/probes/encode_probe.py > gpurun_out/enc_$v.log 2>&1 || { echo "FAILED $v"; tail -20 gpurun_out/enc_$v.log; exit 1; }
  echo "== $v"; grep encode gpurun_out/enc_$v.log
  f=$(find /tmp/pe_$v -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r.get("Name", r.get("KernelName", "?"))
    if "topk" in n:
        print(f"  {n[:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:7.2f} us")
PY
done
