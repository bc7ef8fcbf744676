#!/bin/bash
# Round-5 batch 24: k_hconv with the tap loop kept rolled (PDE_HCONV_V=1: no hoisted 9-tap address
# table, 16 fragment reads up front) vs the unrolled form (0): conv / ResNet GPU tests, per-layer conv
# timings and ResNet-18 benches, interleaved.  VARIANTS="0 1 2" picks the forms, NO_RN=1 skips the benches.
set -o pipefail
O=gpurun_out/${1:-r5_b24}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for v in ${VARIANTS:-0 1}; do
    PDE_HCONV_V=$v timeout -k 10 300 python tools/conv_bench.py --stages 2 > $O/conv_v${v}_$r.jsonl 2> $O/conv.err \
      || { tail -20 $O/conv.err; exit 1; }
    python - $O/conv_v${v}_$r.jsonl $v <<'PY'
import json, sys
out = []
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "fprop_us" in d and d["layer"] in ("l2.conv", "l3.conv", "l4.conv", "l1.conv"):
        out.append(f'{d["layer"]} {d["fprop_us"]}/{d["dgrad_us"]}')
print("v", sys.argv[2], " ".join(out))
PY
  done
done
[ -n "$NO_RN" ] && exit 0
for r in 1 2; do
  for v in ${VARIANTS:-0 1}; do
    PDE_HCONV_V=$v timeout -k 10 400 python bench.py --model resnet18 --steps 30 --warmup 5 --comm-figure off \
      > $O/rn_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "v $v rep $r: $(python -c "import json;d=json.load(open('$O/rn_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
