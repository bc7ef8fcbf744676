#!/bin/bash
# Round-5 batch 3: continuous persistent GEMM (cfg 20) + in-place peer all-reduce: GPU tests, the W=1
# comm figure (route timings on the registered flat gradient buffer), GEMM fprop / dgrad timings.
set -o pipefail
O=gpurun_out/${1:-r5_b3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
  -k "gemm8pc or gemm8pp or schedules_match or persistent_multi_tile or tiles_and_cfgs or peer_inplace or peer_allreduce_matches or peer_engine" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_comm.json 2> $O/bench_comm.err || exit 1
# HIP runtime knobs on the headline step (kernel arguments in device memory, graph packet capture)
for r in 1 2; do
  for e in NONE=1 HIP_FORCE_DEV_KERNARG=1 HIP_FORCE_DEV_KERNARG=0 DEBUG_CLR_GRAPH_PACKET_CAPTURE=0; do
    env $e timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/env_${e}_$r.json 2>> $O/env.err || exit 1
  done
done
timeout -k 10 300 python tools/gemm_own_bench.py --only fprop,dgrad --cfgs 16,18,19,20,21 > $O/gemm.jsonl 2> $O/gemm.err || exit 1
python - $O <<'PY'
import json, sys, glob, os
o = sys.argv[1]
d = json.load(open(os.path.join(o, "bench_comm.json")))
w = d.get("w1_rccl_comm", {})
print("headline", d["value"], d["ms_per_step"])
print("comm", w.get("ms_per_step"), w.get("schedule"), w.get("compute_only_us_per_step"), w.get("peer_inplace"), w.get("error"))
print("routes", json.dumps(w.get("route_us_per_call")))
print("scheds", json.dumps(w.get("schedule_us_per_step")))
PY
for f in $O/env_*.json; do echo "$(basename $f) $(python -c "import json;print(json.load(open('$f'))['ms_per_step'])")"; done
cat $O/gemm.jsonl
exit $TRC
