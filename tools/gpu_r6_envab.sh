#!/bin/bash
# Round 6: same-box A/B of one build under an environment switch (ENV=name, values $2 = "old" value and
# $3 = "new" value): LeNet GPU tests, then the toy-CNN headline (driver flags, 5 interleaved reps), the
# 2000-step run (2 reps) and one in-step phase timeline per arm.
#   bash tools/gpu_r6_envab.sh OUTDIR VAR OLDVAL NEWVAL
set -o pipefail
O=gpurun_out/${1:-r6_envab}
VAR=$2; A=$3; B=$4
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_lenet_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3 4 5; do
  for v in old new; do
    val=$A; [ $v = new ] && val=$B
    env $VAR=$val timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/w20_${v}_$r.json 2>> $O/err.txt || exit 1
  done
done
for r in 1 2; do
  for v in old new; do
    val=$A; [ $v = new ] && val=$B
    env $VAR=$val timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/w2000_${v}_$r.json 2>> $O/err.txt || exit 1
  done
done
for v in old new; do
  val=$A; [ $v = new ] && val=$B
  env $VAR=$val timeout -k 10 180 python tools/lenet_phases.py --reps 5 > $O/phases_$v.txt 2>&1 || exit 1
done
python3 - $O <<'PY'
import json, sys, glob, statistics
o = sys.argv[1]
for w in ("w20", "w2000"):
    for v in ("old", "new"):
        xs = [json.load(open(f))["ms_per_step"] * 1000 for f in sorted(glob.glob(f"{o}/{w}_{v}_*.json"))]
        print(w, v, [round(x, 2) for x in xs], "median", round(statistics.median(xs), 2))
PY
grep -h conv_bwd $O/phases_old.txt $O/phases_new.txt | cut -c1-400
