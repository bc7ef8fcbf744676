#!/bin/bash
# Same-box interleaved A/B of the GPT-2 bench: the default GEMM table vs PDE_GEMM_CFG=<B spec>, 3 reps.
# usage: bash tools/gpu_gpt2_ab.sh <tag> '<B spec>'   (e.g. 'fprop:3072:768=15')
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-gpt2ab}
mkdir -p $O
export TMPDIR=/tmp
: > $O/ab.txt
for r in 1 2 3; do
  for arm in A B; do
    spec=""; [ $arm = B ] && spec="$2"
    PDE_GEMM_CFG="$spec" timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/$arm.$r.json 2> $O/$arm.$r.err || { tail -20 $O/$arm.$r.err; exit 1; }
    python3 -c "import json; d=json.load(open('$O/$arm.$r.json')); print('$arm rep $r', d['ms_per_step'], 'ms', d['value'])" >> $O/ab.txt
  done
done
cat $O/ab.txt
