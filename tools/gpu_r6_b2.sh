#!/bin/bash
# Round 6 batch 2: peer tests incl. W = 8 ranks time-sharing the GPU, W2-vs-W1 equivalence (sgd / adam),
# the N = 8 shared-GPU toy-CNN bench rehearsal, then the store-ordering construction + mode timing and
# the persistent-GEMM tests.
set -o pipefail
O=gpurun_out/${1:-r6_b2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 170 python -u -m pytest -x -q -rA --timeout 150 --timeout-method thread tests/test_peer_gpu.py -k "w2_matches" > $O/pytest_w2.txt 2>&1
echo "w2 rc=$?" >> $O/pytest_w2.txt
for t in "inplace_registered_matches_exact and 8-f32" "inplace_registered_matches_exact and 8-bf16" "matches_fp64 and 8"; do
  timeout -k 10 170 python -u -m pytest -x -q -rA --timeout 150 --timeout-method thread tests/test_peer_gpu.py -k "$t" >> $O/pytest_peer8.txt 2>&1 || exit 1
done
PDE_PEER_TIMEOUT_MS=60000 timeout -k 10 420 python bench.py --gpus 8 --shared-gpu --steps 20 --warmup 5 > $O/lenet_n8.json 2> $O/lenet_n8.err
echo "n8 rc=$?" >> $O/lenet_n8.err
timeout -k 10 600 python -u tools/gemm_store_order.py --reps 8 > $O/store_order.jsonl 2> $O/store_order.err || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_gpu.py -k "gemm8pp or gemm8pc or persistent or dgrad" > $O/pytest_gemm.txt 2>&1 || exit 1
tail -3 $O/pytest_gemm.txt
