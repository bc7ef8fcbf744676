#!/bin/bash
# Round-3 iteration: LeNet + transformer GPU tests, headline A/B vs the round-2 worktree, GPT-2 bench
# and its step-window kernel table.
set -o pipefail
O=gpurun_out/${1:-iter}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_lenet_gpu.py tests/test_transformer_gpu.py tests/test_gemm_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -4 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ${1:-iter}/ab || exit 1
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || exit 1
python -c "import json;d=json.load(open('$O/bench_gpt2.json'));print('gpt2', d['value'], d['ms_per_step'])"
