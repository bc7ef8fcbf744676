#!/bin/bash
# Round-5 batch 21: same-box A/B of the halo image layout (PDE_HALO_KEY=1 key-swizzled, 0 row-swizzled):
# conv tests under both, per-layer conv timings and ResNet-18 benches interleaved.
set -o pipefail
O=gpurun_out/${1:-r5_b21}
mkdir -p $O
export TMPDIR=/tmp
PDE_HALO_KEY=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  > $O/pytest_key0.txt 2>&1 || { tail -40 $O/pytest_key0.txt; exit 1; }
tail -1 $O/pytest_key0.txt
for r in 1 2; do
  for v in 1 0; do
    PDE_HALO_KEY=$v timeout -k 10 300 python tools/conv_bench.py --stages 2 > $O/conv_k${v}_$r.jsonl 2> $O/conv.err || { tail -20 $O/conv.err; exit 1; }
    python - $O/conv_k${v}_$r.jsonl "key=$v rep $r" <<'PY'
import json, sys
out = []
for l in open(sys.argv[1]):
    d = json.loads(l)
    if d.get("layer") in ("l2.conv", "l3.conv"):
        out.append(f'{d["layer"]} f {d["fprop_us"]} d {d["dgrad_us"]}')
print(sys.argv[2], " | ".join(out))
PY
  done
done
for r in 1 2; do
  for v in 1 0; do
    PDE_HALO_KEY=$v timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off > $O/rn_k${v}_$r.json 2>> $O/err.txt \
      || { tail -20 $O/err.txt; exit 1; }
    echo "key=$v rep $r: $(python -c "import json;d=json.load(open('$O/rn_k${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
