#!/bin/bash
# Round 6 end: smoke() and the driver's two bench invocations (no flags; --gpus 1 --steps 20 --warmup 5).
set -o pipefail
O=gpurun_out/${1:-r6_final2}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_default", "bench_driver"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d["value"], d["ms_per_step"], d["steps"], d["warmup"], d["config"]["mode"], d["config"]["host_cpus"],
          d.get("w1_rccl_comm", {}).get("ms_per_step"))
PY
