#!/bin/bash
# Round-5 batch 10: route timings as graph-replayed GPU time (default) vs eager launches; peer GPU tests.
# (The batch also ran a cross-entropy non-temporal A/B whose code was reverted: profiles/r5_gpt2/rejected_xent_nt/.)
set -o pipefail
O=gpurun_out/${1:-r5_b10}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread tests/test_peer_gpu.py \
  > $O/pytest_peer.txt 2>&1 || { tail -30 $O/pytest_peer.txt; exit 1; }
tail -2 $O/pytest_peer.txt
for m in graph eager graph; do
  PDE_ROUTE_TIMING=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/lenet_$m.json 2> $O/lenet_$m.err || exit 1
  python - $O/lenet_$m.json $m <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); w = d.get("w1_rccl_comm", {})
print(sys.argv[2], "headline", d["ms_per_step"], "| comm", w.get("ms_per_step"), w.get("schedule"),
      "compute", w.get("compute_only_us_per_step"), "routes", json.dumps(w.get("route_us_per_call")))
PY
done
