#!/bin/bash
# Full GPU suite + smoke + driver-config benches (headline with its W=1 comm figure, 2000-step headline,
# GPT-2, ResNet-18), one box.
set -o pipefail
O=gpurun_out/${1:-r4_full}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --maxfail=20 --timeout 170 --timeout-method thread > $O/pytest_gpu.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest_gpu.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest_gpu.txt | cut -c1-300; tail -2 $O/pytest_gpu.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { cat $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/bench_long.json 2> $O/bench_long.err || exit 1
timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || exit 1
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err || exit 1
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_driver", "bench_long", "bench_gpt2", "bench_resnet18"):
    d = json.load(open(f"{o}/{f}.json"))
    w = d.get("w1_rccl_comm", {})
    print(f, d["value"], d["ms_per_step"], "| comm:", w.get("value"), w.get("ms_per_step"), w.get("schedule", w.get("mode")),
          d["config"].get("compute_only_us_per_step", w.get("compute_only_us_per_step")))
PY
exit $TRC
