#!/bin/bash
# Round 6: persistent-GEMM store ordering -- correctness per mode (incl. the failure construction), timing
# per mode on the GPT-2 shapes, the persistent-GEMM GPU tests, and GPT-2 benches with dgrad on cfg 18 / 19.
set -o pipefail
O=gpurun_out/${1:-r6_gemm}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/gemm_store_order.py --reps ${REPS:-5} > $O/store_order.jsonl 2> $O/store_order.err || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "gemm8pp or gemm8pc or persistent or dgrad" > $O/pytest_gemm.txt 2>&1 || exit 1
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_table.json 2> $O/gpt2_table.err || exit 1
PDE_GEMM_CFG="dgrad:768:3072=19,dgrad:3072:768=19,dgrad:768:50304=19" timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_dgrad19.json 2> $O/gpt2_dgrad19.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_lenet.json 2> $O/bench_lenet.err || exit 1
tail -3 $O/pytest_gemm.txt
for f in gpt2_table gpt2_dgrad19 bench_lenet; do python -c "import json,sys; d=json.load(open('$O/$f.json')); print('$f', d['value'], d['ms_per_step'])"; done
