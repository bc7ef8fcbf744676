#!/bin/bash
# Full-state check: all GPU tests, smoke, headline bench + GPT-2 / ResNet-18 benches.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; r=$?
tail -4 gpurun_out/pytest_gpu.log
[ $r -le 1 ] || exit $r
timeout -k 10 300 python __graft_entry__.py smoke > gpurun_out/smoke.log 2>&1 && tail -1 gpurun_out/smoke.log &&
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cat gpurun_out/bench_default.json &&
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 > gpurun_out/bench_graph.json 2> gpurun_out/bench_graph.err && cat gpurun_out/bench_graph.json &&
timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.err && cat gpurun_out/bench_gpt2.json &&
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/bench_resnet18.json 2> gpurun_out/bench_resnet18.err && cat gpurun_out/bench_resnet18.json
rc=$?
grep -E "FAILED|ERROR" gpurun_out/pytest_gpu.log | head -20
echo "pytest_rc=$r rc=$rc"
exit $rc
