#!/bin/bash
# Interleaved A/B of the headline bench on ONE box: _r2base (baseline worktree, built in-tree) vs the
# current tree (optionally with an env assignment for B), driver config (20/5) and a long run.
# usage: tools/gpu_ab.sh OUT [ENV=VALUE]
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in base new; do
    if [ $v = base ]; then D=_r2base; E=""; else D=.; E="$2"; fi
    (cd $D && env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off) > $O/$v$rep.json 2> $O/$v$rep.err || exit 1
    (cd $D && env $E timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --comm-figure off) > $O/${v}L$rep.json 2> $O/${v}L$rep.err || exit 1
    python -c "import json;print('$v', json.load(open('$O/$v$rep.json'))['ms_per_step'], 'long', json.load(open('$O/${v}L$rep.json'))['ms_per_step'])"
  done
done
