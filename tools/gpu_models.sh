#!/bin/bash
# GPU session for the driver-added model configs: tests + short benches (+ optional rocprof).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STAGE=${1:-all}
tests() { timeout -k 10 900 python -m pytest tests/test_resnet_gpu.py tests/test_transformer_gpu.py -q -x > gpurun_out/pytest_models.log 2>&1; r=$?; tail -30 gpurun_out/pytest_models.log; [ $r -le 1 ]; }
bench_rn() { timeout -k 10 400 python bench.py --model resnet18 --steps ${STEPS:-20} --warmup 5 > gpurun_out/bench_resnet18.json 2> gpurun_out/bench_resnet18.err; r=$?; cat gpurun_out/bench_resnet18.json; tail -5 gpurun_out/bench_resnet18.err; return $r; }
bench_gpt() { timeout -k 10 400 python bench.py --model gpt2 --steps ${STEPS:-20} --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.err; r=$?; cat gpurun_out/bench_gpt2.json; tail -5 gpurun_out/bench_gpt2.err; return $r; }
prof_rn() { timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_rn" -o rn -- python3 bench.py --model resnet18 --steps 5 --warmup 2 > gpurun_out/prof_rn.log 2>&1; }
prof_gpt() { timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_gpt2" -o gpt2 -- python3 bench.py --model gpt2 --steps 5 --warmup 2 > gpurun_out/prof_gpt2.log 2>&1; }
case "$STAGE" in
  tests) tests ;;
  rn) tests && bench_rn && prof_rn ;;
  gpt) bench_gpt && prof_gpt ;;
  all) tests && bench_rn && bench_gpt && prof_rn && prof_gpt ;;
esac
rc=$?
echo "stage=$STAGE rc=$rc"
exit $rc
