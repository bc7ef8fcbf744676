#!/bin/bash
# Round-5 start: driver-config benches of the three models + own-vs-library GEMM fprop timings.
set -o pipefail
O=gpurun_out/${1:-r5_base}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || exit 1
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err || exit 1
timeout -k 10 300 python tools/gemm_own_bench.py --only fprop --cfgs 9,17,18 > $O/gemm_fprop.jsonl 2> $O/gemm.err || exit 1
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_driver", "bench_gpt2", "bench_resnet18"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d["value"], d["ms_per_step"])
PY
cat $O/gemm_fprop.jsonl
