#!/bin/bash
# Round 6 batch 3: kernel timeline of the W=1 comm-path step per schedule (compute-only, serial peer1,
# overlap2 peer1/rccl), and own-GEMM fprop / dgrad timings per config at the GPT-2 shapes.
set -o pipefail
O=gpurun_out/${1:-r6_b3}
mkdir -p $O
export TMPDIR=/tmp
for s in "none" "serial 431296:peer1" "overlap2 25664:peer1,405632:rccl" "serial 431296:rccl"; do
  tag=$(echo "$s" | tr ' :,' '___')
  timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/tr_$tag" -o tr \
    -- python3 bench.py --steps 400 --warmup 20 --force-comm --schedule "$s" --comm-figure off > $O/tr_$tag.json 2> $O/tr_$tag.err || exit 1
  f=$(find $O/tr_$tag -name "*kernel_trace.csv" | head -1)
  echo "== $s  $(python3 -c "import json; d=json.load(open('$O/tr_$tag.json')); print(d['ms_per_step'])")" >> $O/timelines.txt
  python3 tools/trace_summary.py "$f" k_conv_fwd2 10 >> $O/timelines.txt || exit 1
  rm -f "$f"
done
timeout -k 10 400 python tools/gemm_own_bench.py --only fprop,dgrad --cfgs 9,16,18,19,20,22 --iters 20 > $O/gemm_own.jsonl 2> $O/gemm_own.err || exit 1
cat $O/timelines.txt
