#!/bin/bash
# One GPU-box session: numerics tests, smoke, bench (graph + eager), rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps chained with && so the first failure ends the call.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
# pytest rc 1 (= some test failed) still lets the later stages run; a crash / timeout (other rc) stops.
run_tests() { timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; r=$?; [ $r -le 1 ]; }
run_smoke() { timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1; }
run_bench() {
  timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err &&
  timeout -k 10 300 python bench.py --steps 1000 --warmup 100 --mode eager > gpurun_out/bench_eager.json 2> gpurun_out/bench_eager.err
}
run_prof() {
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof" -o lenet \
    -- python3 bench.py --steps 300 --warmup 20 > gpurun_out/prof.log 2>&1
}
run_kbench() { timeout -k 10 300 python tools/kbench_lenet.py > gpurun_out/kbench.log 2>&1; }
run_pmc() {
  rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || true
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/pmc" -o lenet \
    --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE \
    -- python3 bench.py --steps 50 --warmup 5 --mode eager > gpurun_out/pmc.log 2>&1
}
case "$STAGE" in
  kbench) run_kbench ;;
  pmc) run_pmc ;;
  kb_pmc) run_kbench && run_pmc ;;
  tests) run_tests ;;
  bench) run_bench ;;
  prof) run_prof ;;
  all) run_tests && run_smoke && run_bench && run_prof ;;
  nobench) run_tests && run_smoke ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc"
tail -3 gpurun_out/pytest_gpu.log 2>/dev/null
cat gpurun_out/smoke.log gpurun_out/bench_*.json 2>/dev/null | tail -5
cat gpurun_out/kbench.log 2>/dev/null | tail -30
exit $rc
