#!/bin/bash
# Round 6 batch 4: the fused fold + all-reduce route ("serial ...:pfold"): bit-identity tests at W = 1 / 2 / 4,
# kernel timeline, the W=1 comm figure with it among the autotuned schedules; GPT-2 table A/B.
set -o pipefail
O=gpurun_out/${1:-r6_b4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 170 python -u -m pytest -x -q -rA --timeout 150 --timeout-method thread tests/test_peer_gpu.py -k "pfold" > $O/pytest_pfold.txt 2>&1 || exit 1
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/tr_pfold" -o tr \
  -- python3 bench.py --steps 400 --warmup 20 --force-comm --schedule "serial 431296:pfold" --comm-figure off > $O/tr_pfold.json 2> $O/tr_pfold.err || exit 1
f=$(find $O/tr_pfold -name "*kernel_trace.csv" | head -1)
python3 tools/trace_summary.py "$f" k_conv_fwd2 10 > $O/timeline_pfold.txt || exit 1
rm -f "$f"
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || exit 1
done
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_A.json 2> $O/gpt2_A.err || exit 1
PDE_GEMM_CFG="fprop:2304:768=22,dgrad:768:2304=19" timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_B.json 2> $O/gpt2_B.err || exit 1
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_A2.json 2> $O/gpt2_A2.err || exit 1
PDE_GEMM_CFG="fprop:2304:768=22,dgrad:768:2304=19" timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_B2.json 2> $O/gpt2_B2.err || exit 1
timeout -k 10 400 python tools/gemm_own_bench.py --only dgrad --cfgs 18,19 --iters 20 > $O/gemm_dgrad_split.jsonl 2> $O/gemm_dgrad_split.err || exit 1
cat $O/timeline_pfold.txt
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_1", "bench_2", "gpt2_A", "gpt2_B", "gpt2_A2", "gpt2_B2"):
    d = json.load(open(f"{o}/{f}.json"))
    c = d.get("w1_rccl_comm", {})
    print(f, d["value"], d["ms_per_step"], c.get("schedule"), c.get("ms_per_step"), c.get("compute_only_us_per_step"))
PY
