#!/bin/bash
# Round-5 batch 11: in-place peer all-reduce with the call count in barrier A's atomic signal, bf16
# in-place form, DDP flat gradients registered: peer GPU tests, W=1 route timings, GPT-2 / ResNet W=1
# comm figures (DDP peer route in place).
set -o pipefail
O=gpurun_out/${1:-r5_b11}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 170 --timeout-method thread tests/test_peer_gpu.py \
  > $O/pytest_peer.txt 2>&1 || { tail -40 $O/pytest_peer.txt; exit 1; }
tail -2 $O/pytest_peer.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/lenet.json 2> $O/lenet.err || exit 1
python - $O/lenet.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); w = d.get("w1_rccl_comm", {})
print("lenet headline", d["ms_per_step"], "| comm", w.get("ms_per_step"), w.get("schedule"),
      "compute", w.get("compute_only_us_per_step"), "routes", json.dumps(w.get("route_us_per_call")))
PY
for m in gpt2 resnet18; do
  timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 > $O/$m.json 2> $O/$m.err || exit 1
  python - $O/$m.json $m <<'PY'
import json, sys
d = json.load(open(sys.argv[1])); w = d.get("w1_rccl_comm", {})
print(sys.argv[2], d["value"], d["ms_per_step"], "| comm", w.get("value"), w.get("ms_per_step"), w.get("grad_reduce_route"),
      "inplace", w.get("peer_inplace"), "bucket", w.get("bucket_mb"))
PY
done
