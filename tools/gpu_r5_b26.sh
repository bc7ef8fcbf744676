#!/bin/bash
# Round-5 batch 26: k_hconv64 with a tap's 12 fragment reads issued ahead of its 8 MFMAs (PDE_HC64_PIPE=1)
# vs interleaved with them (0): conv / ResNet GPU tests, layer-1 conv timings, ResNet-18 benches, interleaved.
set -o pipefail
O=gpurun_out/${1:-r5_b26}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for v in 0 1; do
    PDE_HC64_PIPE=$v timeout -k 10 300 python tools/conv_bench.py --stages 2 > $O/conv_i${v}_$r.jsonl 2> $O/conv.err \
      || { tail -20 $O/conv.err; exit 1; }
    python - $O/conv_i${v}_$r.jsonl $v <<'PY'
import json, sys
out, tot = [], 0.0
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "fprop_us" in d and d["layer"] == "l1.conv":
        out.append(f'{d["layer"]} fprop {d["fprop_us"]} dgrad {d["dgrad_us"]} wgrad {d["wgrad_us"]}')
print("pipe", sys.argv[2], " ".join(out))
PY
  done
done
for r in 1 2; do
  for v in 0 1; do
    PDE_HC64_PIPE=$v timeout -k 10 400 python bench.py --model resnet18 --steps 30 --warmup 5 --comm-figure off \
      > $O/rn_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "pipe $v rep $r: $(python -c "import json;d=json.load(open('$O/rn_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
