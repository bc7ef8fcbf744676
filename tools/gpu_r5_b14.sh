#!/bin/bash
# Round-5 batch 14: the N>1 bench path rehearsed with ranks sharing one GPU (gloo control plane, xGMI
# peer kernel for every collective): toy CNN at N=2 and N=4, GPT-2 and ResNet-18 at N=2.
set -o pipefail
O=gpurun_out/${1:-r5_b14}
mkdir -p $O
export TMPDIR=/tmp
for n in ${LENET_NS-2 4}; do
  timeout -k 10 400 python bench.py --gpus $n --shared-gpu --steps 20 --warmup 5 > $O/lenet_n$n.json 2> $O/lenet_n$n.err \
    || { tail -30 $O/lenet_n$n.err; exit 1; }
  python - $O/lenet_n$n.json <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
keep = {k: d.get(k) for k in ("value", "ms_per_step", "n_gpus", "w1_anchor_images_per_s", "scaling_eff_same_job")}
c = d.get("config", {})
print(json.dumps(keep), "schedule", c.get("schedule"), "routes", json.dumps(c.get("route_us_per_call")))
print("per_rank", json.dumps(d.get("per_rank"))[:400])
PY
done
for m in gpt2 resnet18; do
  timeout -k 10 500 python bench.py --model $m --gpus 2 --shared-gpu --steps 10 --warmup 3 > $O/${m}_n2.json 2> $O/${m}_n2.err \
    || { tail -30 $O/${m}_n2.err; exit 1; }
  python -c "import json;d=json.load(open('$O/${m}_n2.json'));print('$m', d['value'], d['ms_per_step'], json.dumps(d.get('config',{}))[:600])"
done
