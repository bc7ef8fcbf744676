#!/bin/bash
# Round-5 batch 20: key-swizzled halo image in k_hconv: conv / ResNet GPU tests, per-layer conv timings,
# ResNet-18 benches, bank-conflict PMC of the halo convolutions.
set -o pipefail
O=gpurun_out/${1:-r5_b20}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 300 python tools/conv_bench.py --stages 2 > $O/conv.jsonl 2> $O/conv.err || { tail -20 $O/conv.err; exit 1; }
python - $O/conv.jsonl <<'PY'
import json, sys
tf = td = 0.0
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "fprop_us" in d:
        tf += d["fprop_us"] * d["count"]; td += d["dgrad_us"] * d["count"]
        print(d["layer"], "fprop", d["fprop_us"], "dgrad", d["dgrad_us"], "wgrad", d["wgrad_us"])
print("fprop total", round(tf, 1), "dgrad total", round(td, 1))
PY
for r in 1 2; do
  timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off > $O/rn_$r.json 2>> $O/err.txt \
    || { tail -20 $O/err.txt; exit 1; }
  echo "rep $r: $(python -c "import json;d=json.load(open('$O/rn_$r.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/pmc" -o rn --pmc SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS \
  -- python3 bench.py --model resnet18 --steps 2 --warmup 1 --model-graph off --comm-figure off > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
python3 tools/pmc_pick.py $O "k_hconv<" k_hconv64 > $O/pmc_pick.txt && cat $O/pmc_pick.txt
