#!/bin/bash
# Round 6 batch 3: the store-ordering construction (decoys spread per block) vs round 5's allowance,
# the GEMM + cross-entropy GPU tests, kernel timelines of the W=1 comm-path step per schedule, GPT-2 with
# the round-6 dgrad table, and the N = 8 shared-GPU rehearsal with its wall time.
set -o pipefail
O=gpurun_out/${1:-r6_b3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/gemm_store_order.py --modes 1,2 --reps 10 --skip-timing > $O/store_order_c.jsonl 2> $O/store_order_c.err || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py > $O/pytest_gemm.txt 2>&1 || exit 1
timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_gpu.py -k xent > $O/pytest_xent.txt 2>&1 || exit 1
for s in "none" "serial 431296:peer1" "overlap2 25664:peer1,405632:rccl" "serial 431296:rccl"; do
  tag=$(echo "$s" | tr ' :,' '___')
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/tr_$tag" -o tr \
    -- python3 bench.py --steps 400 --warmup 20 --force-comm --schedule "$s" --comm-figure off > $O/tr_$tag.json 2> $O/tr_$tag.err || exit 1
  f=$(find $O/tr_$tag -name "*kernel_trace.csv" | head -1)
  echo "== $s  $(python3 -c "import json; d=json.load(open('$O/tr_$tag.json')); print(d['ms_per_step'])")" >> $O/timelines.txt
  python3 tools/trace_summary.py "$f" k_conv_fwd2 10 >> $O/timelines.txt || exit 1
  rm -f "$f"
done
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2.json 2> $O/gpt2.err || exit 1
t0=$(date +%s)
PDE_PEER_TIMEOUT_MS=60000 timeout -k 10 420 python bench.py --gpus 8 --shared-gpu --steps 20 --warmup 5 > $O/lenet_n8.json 2> $O/lenet_n8.err
echo "n8 rc=$? wall_s=$(( $(date +%s) - $t0 ))" >> $O/lenet_n8.err
timeout -k 10 400 python tools/gemm_own_bench.py --only fprop,dgrad --cfgs 9,16,18,19,22 --iters 20 > $O/gemm_own.jsonl 2> $O/gemm_own.err || exit 1
cat $O/timelines.txt
