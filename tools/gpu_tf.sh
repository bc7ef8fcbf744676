#!/bin/bash
# GPU session for the transformer stack: kernel/model tests, then a short GPT-2 bench + rocprof stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
tests() { timeout -k 10 600 python -m pytest tests/test_transformer_gpu.py -q -x > gpurun_out/pytest_tf.log 2>&1; r=$?; tail -30 gpurun_out/pytest_tf.log; [ $r -le 1 ]; }
bench() { timeout -k 10 400 python bench.py --model gpt2 --steps ${STEPS:-20} --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.err; r=$?; cat gpurun_out/bench_gpt2.json; tail -5 gpurun_out/bench_gpt2.err; return $r; }
prof() { timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_gpt2" -o gpt2 -- python3 bench.py --model gpt2 --steps 5 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1; }
case "$STAGE" in
  tests) tests ;;
  bench) bench ;;
  prof) prof ;;
  all) tests && bench && prof ;;
  tb) tests && bench ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc"
exit $rc
