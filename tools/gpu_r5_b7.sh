#!/bin/bash
# Round-5 batch 7: dgrad tile configs (best of two timings), GPT-2 with the final table, the toy-CNN W=1
# comm figure (in-place peer routes, overlap2), ResNet-18 reference run.
set -o pipefail
O=gpurun_out/${1:-r5_b7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python tools/gemm_own_bench.py --only dgrad --cfgs 9,16,18,19 > $O/gemm_dgrad.jsonl 2> $O/gemm.err || exit 1
cat $O/gemm_dgrad.jsonl
for r in 1 2; do
  timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_$r.json 2>> $O/err.txt || exit 1
  echo "gpt2 rep $r: $(python -c "import json;d=json.load(open('$O/gpt2_$r.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/lenet.json 2> $O/lenet.err || exit 1
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/resnet18.json 2> $O/resnet18.err || exit 1
python - $O <<'PY'
import json, sys, os
o = sys.argv[1]
d = json.load(open(os.path.join(o, "lenet.json")))
w = d.get("w1_rccl_comm", {})
print("lenet", d["value"], d["ms_per_step"], "| comm", w.get("ms_per_step"), w.get("schedule"), w.get("compute_only_us_per_step"), w.get("peer_inplace"))
print("routes", json.dumps(w.get("route_us_per_call")))
print("scheds", json.dumps(w.get("schedule_us_per_step")))
r = json.load(open(os.path.join(o, "resnet18.json")))
print("resnet18", r["value"], r["ms_per_step"])
PY
