#!/bin/bash
# Round 6 end: the driver's default bench invocation, an N = 2 rehearsal on one time-shared GPU, and
# GPT-2 / ResNet-18 runs of the final bench.py (NUMA pinning on).
set -o pipefail
O=gpurun_out/${1:-r6_final_bench}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench_default.json 2> $O/bench_default.err || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || exit 1
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29613 bench.py --gpus 2 --shared-gpu --steps 20 --warmup 5 > $O/bench_n2_shared.json 2> $O/bench_n2_shared.err || exit 1
timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || exit 1
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err || exit 1
python3 - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("bench_default", "bench_driver", "bench_n2_shared", "bench_gpt2", "bench_resnet18"):
    d = json.load(open(f"{o}/{f}.json"))
    print(f, d.get("value"), d.get("ms_per_step"), d.get("n_gpus"), d["config"].get("host_cpus"), d["config"].get("parallelism"))
PY
