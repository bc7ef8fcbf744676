#!/bin/bash
# Same-box A/B of one environment switch on the headline step: phase timeline + driver-config bench
# + 2000-step bench for the default tree and with "$2" exported (e.g. PDE_LENET_HEAD=1), 2 reps each.
# usage: bash tools/gpu_ab_env.sh <tag> <VAR=value> [pytest -k expr]
set -o pipefail
O=gpurun_out/${1:-ab}
ENVB=$2
K=$3
mkdir -p $O
export TMPDIR=/tmp
TRC=0
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -k "$K" > $O/pytest.txt 2>&1
  TRC=$?
  # 0 = passed, 1 = some tests failed (assertions): go on with the A/B; anything else (a crash, a
  # time-out, an abort) ends this GPU call here
  if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
  grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300
  tail -3 $O/pytest.txt
fi
timeout -k 10 200 python tools/lenet_phases.py --reps 5 > $O/phases_A.txt 2>&1 &&
env $ENVB timeout -k 10 200 python tools/lenet_phases.py --reps 5 > $O/phases_B.txt 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/A20_$r.json 2>> $O/err.txt &&
  env $ENVB timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/B20_$r.json 2>> $O/err.txt &&
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/A2000_$r.json 2>> $O/err.txt &&
  env $ENVB timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/B2000_$r.json 2>> $O/err.txt || exit 1
done
python - $O <<'PY'
import json, sys, glob, os
o = sys.argv[1]
for f in sorted(glob.glob(os.path.join(o, "*.json"))):
    try:
        print(os.path.basename(f), json.load(open(f))["ms_per_step"])
    except Exception as e:
        print(f, "ERR", e)
PY
grep -h "^head\|^fc_bwd\|^adam\|^conv_bwd" $O/phases_A.txt $O/phases_B.txt | cut -c1-200
exit $TRC
