#!/bin/bash
# Round-5 batch 2: new GPU tests (persistent 8-phase GEMM, in-place peer all-reduce, advisor fixes),
# Adam non-temporal parameter stores A/B, the W=1 comm figure with in-place peer routes, GEMM fprop timings.
set -o pipefail
O=gpurun_out/${1:-r5_b2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
  -k "gemm8pp or persistent_multi_tile or tiles_and_cfgs or peer_inplace or test_lenet_gpu or peer_buffer or w2_matches or head_no_bias or peer_allreduce_matches" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/ntp1_$r.json 2>> $O/err.txt &&
  PDE_ADAM_NT_P=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/ntp0_$r.json 2>> $O/err.txt || exit 1
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_comm.json 2> $O/bench_comm.err || exit 1
timeout -k 10 300 python tools/gemm_own_bench.py --only fprop,dgrad --cfgs 17,18,19 > $O/gemm.jsonl 2> $O/gemm.err || exit 1
python - $O <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "ntp*.json"))):
    print(os.path.basename(f), json.load(open(f))["ms_per_step"])
d = json.load(open(os.path.join(o, "bench_comm.json")))
w = d.get("w1_rccl_comm", {})
print("headline", d["value"], d["ms_per_step"])
print("comm", w.get("ms_per_step"), w.get("schedule"), w.get("compute_only_us_per_step"), w.get("peer_inplace"))
print("routes", json.dumps(w.get("route_us_per_call")))
print("scheds", json.dumps(w.get("schedule_us_per_step")))
PY
cat $O/gemm.jsonl
exit $TRC
