#!/bin/bash
# Round 6: GPT-2 / ResNet-18 benches (driver flags) with and without the NUMA pinning, interleaved, one box.
set -o pipefail
O=gpurun_out/${1:-r6_models_numa}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for m in resnet18 gpt2; do
    for n in 1 0; do
      PDE_BENCH_NUMA=$n timeout -k 10 300 python bench.py --model $m --steps 20 --warmup 5 --comm-figure off \
        > $O/${m}_numa${n}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    done
  done
done
python3 - $O <<'PY'
import json, sys, glob, statistics
o = sys.argv[1]
for m in ("resnet18", "gpt2"):
    for n in ("1", "0"):
        rows = [json.load(open(f)) for f in sorted(glob.glob(f"{o}/{m}_numa{n}_*.json"))]
        xs = [d["value"] for d in rows]
        print(m, "numa", n, [round(x) for x in xs], "median", round(statistics.median(xs)), rows[0]["config"]["host_cpus"])
PY
