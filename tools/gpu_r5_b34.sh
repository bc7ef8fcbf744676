#!/bin/bash
# Round-5 batch 34: single-exp cross-entropy (k_xent_bf16_reg2, default) vs the online-softmax kernel
# (PDE_XENT_V=1): transformer GPU tests, GPT-2 benches interleaved, a kernel-trace of one short run each.
set -o pipefail
O=gpurun_out/${1:-r5_b34}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_transformer_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2 3; do
  for v in 1 2; do
    PDE_XENT_V=$v timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 --comm-figure off \
      > $O/gpt2_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "xent v$v rep $r: $(python -c "import json;d=json.load(open('$O/gpt2_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for v in 1 2; do
  PDE_XENT_V=$v timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/trace_$v" -o g \
    -- python3 bench.py --model gpt2 --steps 4 --warmup 2 --comm-figure off > $O/trace_$v.log 2>&1 || { tail -5 $O/trace_$v.log; exit 1; }
done
python3 - "$O" <<'PY'
import csv, glob, sys
for v in (1, 2):
    f = glob.glob(f"{sys.argv[1]}/trace_{v}/**/*kernel_stats.csv", recursive=True)[0]
    for r in csv.DictReader(open(f)):
        if "xent" in r["Name"]:
            print(v, r["Name"][:60], "calls", r["Calls"], "avg us", round(float(r["AverageNs"]) / 1e3, 1))
PY
