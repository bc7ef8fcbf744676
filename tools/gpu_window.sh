#!/bin/bash
# Driver-window (20 timed steps) vs steps per captured graph: where the fixed window cost comes from.
set -o pipefail
O=gpurun_out/${1:-window}
mkdir -p $O
export TMPDIR=/tmp PDE_BENCH_TRACE=1
: > $O/window.jsonl
for rep in 1 2; do
  for S in 20 10 5 4 2 1; do
    timeout -k 10 120 python bench.py --steps 20 --warmup 5 --graph-steps $S --comm-figure off > $O/b.json 2> $O/b.err || exit 1
    python - "$S" "$O" <<'PY' >> $O/window.jsonl
import json, sys
S, O = sys.argv[1], sys.argv[2]
b = json.loads(open(f"{O}/b.json").read().strip().splitlines()[-1])
tr = [json.loads(l) for l in open(f"{O}/b.err") if l.startswith('{"trace')]
print(json.dumps({"S": int(S), "us_per_step": round(b["ms_per_step"] * 1e3, 2), **(tr[-1] if tr else {})}))
PY
  done
done
cat $O/window.jsonl
