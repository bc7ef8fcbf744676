#!/bin/bash
# Round-5 batch 18: conv wgrad with the incremental B-row pixel walk (PDE_WGRAD_INCR, default on):
# conv / ResNet GPU tests, per-layer conv timings (both settings), same-box ResNet-18 benches.
set -o pipefail
O=gpurun_out/${1:-r5_b18}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for v in 1 0; do
  PDE_WGRAD_INCR=$v timeout -k 10 300 python tools/conv_bench.py --stages 2 > $O/conv_incr$v.jsonl 2> $O/conv_incr$v.err \
    || { tail -20 $O/conv_incr$v.err; exit 1; }
  python - $O/conv_incr$v.jsonl $v <<'PY'
import json, sys
tot = 0.0
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "wgrad_us" in d:
        tot += d["wgrad_us"] * d["count"]
        print("incr", sys.argv[2], d["layer"], "wgrad", d["wgrad_us"], "us")
print("incr", sys.argv[2], "wgrad total per step", round(tot, 1))
PY
done
for r in 1 2; do
  for v in 1 0; do
    PDE_WGRAD_INCR=$v timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off \
      > $O/rn_i${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "incr=$v rep $r: $(python -c "import json;d=json.load(open('$O/rn_i${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
