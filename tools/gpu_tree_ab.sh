#!/bin/bash
# Same-box A/B of an older tree (a git worktree built in-tree, e.g. _r4a/) against the current tree:
# the given models at the driver's flags, interleaved, 2 reps.
# usage: bash tools/gpu_tree_ab.sh <tag> <base worktree dir> [models...]   (models: lenet gpt2 resnet18)
set -o pipefail
O=gpurun_out/${1:-tree_ab}
BASE=$2
shift 2
M=${@:-resnet18}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for m in $M; do
    for tree in $BASE .; do
      tag=$( [ "$tree" = "." ] && echo cur || echo base )
      (cd $tree && timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 --comm-figure off) > $O/${m}_${tag}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      echo "$m $tag rep $r: $(python -c "import json;d=json.load(open('$O/${m}_${tag}_$r.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
