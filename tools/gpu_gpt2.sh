#!/bin/bash
# GPT-2 iteration: GEMM + transformer GPU tests, the GPT-2 bench (x2) and its step window under rocprofv3.
# usage: bash tools/gpu_gpt2.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-gpt2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gemm_gpu.py tests/test_transformer_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2_$r.json 2> $O/bench_gpt2_$r.err || { tail -20 $O/bench_gpt2_$r.err; exit 1; }
  cut -c1-200 $O/bench_gpt2_$r.json
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o gpt2 -- \
  python3 bench.py --model gpt2 --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof/*kernel_trace.csv | head -n 1)" k_adamw_master 60 > $O/gpt2_step_window.txt
rm -f $O/prof/*kernel_trace.csv
head -40 $O/gpt2_step_window.txt
