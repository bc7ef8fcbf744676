#!/bin/bash
# model tests (transformer + resnet) -> gemm microbench -> resnet/gpt2 benches + resnet profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests/test_resnet_gpu.py tests/test_transformer_gpu.py -q > gpurun_out/pytest_models.log 2>&1; r=$?
tail -25 gpurun_out/pytest_models.log
[ $r -le 1 ] || exit $r
timeout -k 10 300 python tools/gemm_bench.py > gpurun_out/gemm_bench.jsonl 2>&1 && cat gpurun_out/gemm_bench.jsonl &&
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > gpurun_out/bench_resnet18.json 2> gpurun_out/bench_resnet18.err && cat gpurun_out/bench_resnet18.json &&
timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > gpurun_out/bench_gpt2.json 2> gpurun_out/bench_gpt2.err && cat gpurun_out/bench_gpt2.json &&
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_rn" -o rn -- python3 bench.py --model resnet18 --steps 5 --warmup 2 > gpurun_out/prof_rn.log 2>&1
echo "rc=$?"
