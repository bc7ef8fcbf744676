#!/bin/bash
# One-box status pass: driver-style headline bench, GPT-2 / ResNet-18 benches, kernel traces of both
# model steps reduced to step windows, then the whole GPU test suite.
# usage: bash tools/gpu_session.sh <tag> [benches|prof|tests|all]   (default all)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-session}
WHICH=${2:-all}
mkdir -p $O
export TMPDIR=/tmp
benches() {
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
  timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err &&
  timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err
  local r=$?
  cat $O/bench_*.json
  return $r
}
prof() {   # $1 model, $2 tag, $3 step-end kernel
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/$2" -o $2 -- \
    python3 bench.py --model $1 --steps 5 --warmup 2 > $O/$2.log 2>&1 &&
  python3 tools/step_window.py "$(ls $O/$2/*kernel_trace.csv | head -n 1)" "$3" 60 > $O/$2_step_window.txt &&
  rm -f $O/$2/*kernel_trace.csv
}
tests() {
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
  local r=$?
  tail -5 $O/pytest_gpu.txt
  return $r
}
rc=0
case "$WHICH" in
  benches) benches; rc=$? ;;
  prof) prof gpt2 gpt2 k_adamw_master && prof resnet18 rn k_sgd_master; rc=$? ;;
  tests) tests; rc=$? ;;
  all) benches && prof gpt2 gpt2 k_adamw_master && prof resnet18 rn k_sgd_master && tests; rc=$? ;;
esac
head -n 30 $O/*_step_window.txt 2>/dev/null
echo "which=$WHICH rc=$rc"
exit $rc
