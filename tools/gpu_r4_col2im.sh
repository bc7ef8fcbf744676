#!/bin/bash
# Round-4: conv-backward D role with batched LDS reads (col2im gather, conv1 wgrad operands) -- LeNet
# GPU tests, phase timeline, driver-config and 2000-step headline benches.
set -o pipefail
O=gpurun_out/${1:-r4_col2im}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread -k "lenet or engine" > $O/pytest.txt 2>&1
TRC=$?
tail -3 $O/pytest.txt
if [ $TRC -gt 1 ]; then exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300
timeout -k 10 200 python tools/lenet_phases.py --reps 5 > $O/phases.txt 2>&1 || { tail -5 $O/phases.txt; exit 1; }
grep -h "^conv_bwd\|^adam\|^fc_bwd" $O/phases.txt | cut -c1-700
for r in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/w20_$r.json 2>> $O/err.txt || exit 1
done
for r in 1 2; do
  timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/w2000_$r.json 2>> $O/err.txt || exit 1
done
for f in $O/w*.json; do echo "$(basename $f) $(python3 -c "import json;print(json.load(open('$f'))['ms_per_step'])")"; done
exit $TRC
