#!/bin/bash
# Round-5 batch 9: in-place peer all-reduce with per-block call counters (no grid-wide exit atomic):
# peer GPU tests, then the toy-CNN W=1 route timings at 1 / 2 / 4 one-shot vectors per thread.
set -o pipefail
O=gpurun_out/${1:-r5_b9}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_peer_gpu.py \
  > $O/pytest_peer.txt 2>&1 || { tail -30 $O/pytest_peer.txt; exit 1; }
tail -3 $O/pytest_peer.txt
for v in 1 2 4; do
  PDE_PEER_IP_VPT=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/lenet_vpt$v.json 2> $O/lenet_vpt$v.err || exit 1
  python - $O/lenet_vpt$v.json $v <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); w = d.get("w1_rccl_comm", {})
s = w.get("schedule_us_per_step", {})
print("vpt", sys.argv[2], "headline", d["ms_per_step"], "| comm", w.get("ms_per_step"), w.get("schedule"),
      "compute", w.get("compute_only_us_per_step"), "routes", json.dumps(w.get("route_us_per_call")))
PY
done
