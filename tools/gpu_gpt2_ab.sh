#!/bin/bash
# Same-box A/B of GPT-2 bench environment variants: bash tools/gpu_gpt2_ab.sh <tag> "<ENV A>" "<ENV B>" ...
# (use "-" for the default environment); 2 interleaved reps, driver-config bench (20 steps, 5 warm-up).
set -o pipefail
O=gpurun_out/${1:-gpt2ab}
shift
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  i=0
  for e in "$@"; do
    i=$((i+1))
    if [ "$e" = "-" ]; then E=""; else E="$e"; fi
    env $E timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 --comm-figure off > $O/v${i}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "v$i [$e] rep $r: $(python -c "import json;d=json.load(open('$O/v${i}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
