#!/bin/bash
# Interleaved three-way A/B of the headline bench on ONE box: _r2base (baseline worktree), the current
# tree with env A, the current tree with env B; driver config (20/5) and a long run (2000/100).
# usage: tools/gpu_ab3.sh OUT "ENV_A" "ENV_B"
set -o pipefail
O=gpurun_out/${1:-ab3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_lenet_gpu.py -x -q --timeout 200 --timeout-method thread > $O/pytest_lenet.txt 2>&1; rc=$?; tail -3 $O/pytest_lenet.txt; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for v in base A B; do
    case $v in base) D=_r2base; E="";; A) D=.; E="$2";; B) D=.; E="$3";; esac
    (cd $D && env $E timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off) > $O/$v$rep.json 2> $O/$v$rep.err || exit 1
    (cd $D && env $E timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --comm-figure off) > $O/${v}L$rep.json 2> $O/${v}L$rep.err || exit 1
    python -c "import json;print('$v', json.load(open('$O/$v$rep.json'))['ms_per_step'], 'long', json.load(open('$O/${v}L$rep.json'))['ms_per_step'])"
  done
done
