#!/bin/bash
# One parameterised GPU runner for everything this repo measures on an MI355X box.
# Run through gpurun from the repo root, e.g.
#   gpurun --timeout 900 -- bash tools/gpurun_suite.sh tests     # TESTS_K="stem or lazy": a -k filter
#   gpurun --timeout 900 -- bash tools/gpurun_suite.sh bench "--amp none" "--amp bf16"
#   gpurun --timeout 900 -- bash tools/gpurun_suite.sh prof NAME "--amp none --steps 20"
#   gpurun --timeout 900 -- bash tools/gpurun_suite.sh pmc NAME "SQ_WAVES SQ_BUSY_CYCLES" "--amp none"
#   gpurun --timeout 900 -- bash tools/gpurun_suite.sh ab ROUNDS "A|ENV=1|--amp none" "B||--amp none"
#   gpurun --timeout 900 -- bash tools/gpurun_suite.sh validate     # tests + smoke + all presets
# Every GPU step has its own time limit and the first failure ends the script (no retries).
# Outputs land in gpurun_out/ (merged back by gpurun); copy the summaries worth keeping into
# profiles/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 1
export TMPDIR=/tmp
mkdir -p gpurun_out
task=${1:-validate}; shift

run_tests() {
  timeout -k 10 900 python -u -m pytest ${TESTS_ARGS:-tests} -m gpu -x -q --timeout 120 --timeout-method thread \
      ${TESTS_K:+-k "$TESTS_K"} > gpurun_out/gpu_tests.log 2>&1 \
      || { tail -60 gpurun_out/gpu_tests.log; exit 1; }
  tail -1 gpurun_out/gpu_tests.log
}

run_smoke() {
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 \
      || { tail -40 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
}

# bench ARGS...: one bench.py run per argument string, JSON lines appended to gpurun_out/bench.jsonl
run_bench() {
  for args in "$@"; do
    timeout -k 10 400 python bench.py $args > /tmp/bench_out.txt 2> gpurun_out/bench_err.log \
        || { tail -30 gpurun_out/bench_err.log; exit 1; }
    line=$(grep '^{' /tmp/bench_out.txt | tail -1)
    echo "$line" >> gpurun_out/bench.jsonl
    echo "[$args] $(echo "$line" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], "img/s", d["ms_per_step"], "ms", d["dtype"], "enq", d.get("host_enqueue_ms_per_step"))')"
  done
}

# prof NAME ARGS: rocprofv3 kernel trace of bench.py ARGS, summarised over the timed steps
run_prof() {
  name=$1; args=$2
  steps=$(echo "$args" | sed -n 's/.*--steps \([0-9]*\).*/\1/p'); steps=${steps:-20}
  case "$args" in *--steps*) ;; *) args="$args --steps $steps --warmup 6";; esac
  # the headline configuration only: each extra measurement has a timed window of its own, and
  # the summariser's busiest window could be one of theirs (PROF_EXTRAS=1 keeps them)
  [ "${PROF_EXTRAS:-0}" = 1 ] || case "$args" in *--no-extras*) ;; *) args="$args --no-extras";; esac
  rm -rf /tmp/p_$name
  EWDML_PROF_GAP=1 timeout -k 10 600 rocprofv3 --kernel-trace --output-format csv -d /tmp/p_$name \
      -o run -- python3 bench.py $args > gpurun_out/prof_$name.log 2>&1 \
      || { echo "prof $name failed"; tail -30 gpurun_out/prof_$name.log; exit 1; }
  python3 tools/prof_summarize.py /tmp/p_$name gpurun_out/prof_${name}.txt --steps $steps > /dev/null \
      || exit 1
  grep '^{' gpurun_out/prof_$name.log | tail -1
  head -30 gpurun_out/prof_${name}.txt
}

# pmc NAME "COUNTERS" ARGS: one counter pass (respect the per-block limits) over bench.py ARGS
run_pmc() {
  name=$1; counters=$2; args=$3
  rm -rf /tmp/pmc_$name
  timeout -s KILL 300 rocprofv3 --pmc $counters --kernel-trace --output-format csv -d /tmp/pmc_$name \
      -o run -- python3 bench.py $args --steps 5 --warmup 4 > gpurun_out/pmc_$name.log 2>&1 \
      || { echo "pmc $name failed"; tail -30 gpurun_out/pmc_$name.log; exit 1; }
  python3 tools/pmc_summarize.py /tmp/pmc_$name > gpurun_out/pmc_${name}.txt || exit 1
  head -40 gpurun_out/pmc_${name}.txt
}

# ab ROUNDS "NAME|ENV|ARGS"...: interleaved A/B, one line per run in gpurun_out/ab.log
run_ab() {
  rounds=$1; shift
  for r in $(seq 1 "$rounds"); do
    for v in "$@"; do
      IFS='|' read -r name envs args <<< "$v"
      out=$(env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 6 $args 2>/tmp/ab_err.log \
          | grep '^{') || { echo "FAILED $name"; tail -20 /tmp/ab_err.log; exit 1; }
      echo "$name r$r $(echo "$out" | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("host_enqueue_ms_per_step"))')" \
          | tee -a gpurun_out/ab.log
    done
  done
}

# py SCRIPT ARGS: any python tool under its own limit (e.g. tools/methods_eval.py)
run_py() {
  timeout -k 10 ${PY_TIMEOUT:-600} python -u "$@" || exit 1
}

case $task in
  tests) run_tests ;;
  smoke) run_smoke ;;
  bench) run_bench "$@" ;;
  prof) run_prof "$@" ;;
  pmc) run_pmc "$@" ;;
  ab) run_ab "$@" ;;
  py) run_py "$@" ;;
  validate)
    run_tests
    run_smoke
    run_bench "" "--preset lenet" "--preset resnet50_cifar" "--preset resnet50_imagenet" ;;
  *) echo "unknown task $task"; exit 2 ;;
esac
