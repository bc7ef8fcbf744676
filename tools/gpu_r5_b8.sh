#!/bin/bash
# Round-5 batch 8: the toy-CNN W=1 comm figure with / without the in-place peer registration and with
# the peer path off (the timed window of the chosen schedule vs its autotuner time).
set -o pipefail
O=gpurun_out/${1:-r5_b8}
mkdir -p $O
export TMPDIR=/tmp
for e in NONE=1 PDE_PEER_INPLACE=0 PDE_PEER_ALLREDUCE=0; do
  env $e timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/lenet_$e.json 2> $O/lenet_$e.err || exit 1
  python - $O/lenet_$e.json $e <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); w = d.get("w1_rccl_comm", {})
s = w.get("schedule_us_per_step", {})
print(sys.argv[2], "headline", d["ms_per_step"], "| comm", w.get("ms_per_step"), w.get("schedule"),
      "autotune", s.get(w.get("schedule")), "compute", w.get("compute_only_us_per_step"), "overlap2", s.get("overlap2 25664:rccl,405632:rccl"))
PY
done
