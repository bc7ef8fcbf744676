#!/bin/bash
# Round-5 batch 19: stem forward with fixed prefetch offsets and a packed epilogue: conv / ResNet GPU
# tests, ResNet-18 bench, kernel-trace stats of a short ResNet run.
set -o pipefail
O=gpurun_out/${1:-r5_b19}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off > $O/rn_$r.json 2>> $O/err.txt \
    || { tail -20 $O/err.txt; exit 1; }
  echo "rep $r: $(python -c "import json;d=json.load(open('$O/rn_$r.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/trace" -o rn \
  -- python3 bench.py --model resnet18 --steps 10 --warmup 3 --comm-figure off > $O/trace.log 2>&1 || { tail -5 $O/trace.log; exit 1; }
python3 - "$O" <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/trace/**/*kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
for r in rows:
    n = r["Name"]
    if any(k in n for k in ("stem", "k_wgrad<", "hwgrad", "bnpool")):
        print(f'{n[:60]:60s} calls {r["Calls"]:>5s} avg {float(r["AverageNs"])/1e3:8.1f} us')
PY
