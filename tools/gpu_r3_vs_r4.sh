#!/bin/bash
# Same-box A/B of the round-3 tree (git worktree _r3base/, built in-tree) against the current tree:
# ResNet-18, GPT-2 and the headline bench at the driver's flags, interleaved, 2 reps.
# usage: bash tools/gpu_r3_vs_r4.sh <tag> [models...]   (models: lenet gpt2 resnet18)
set -o pipefail
O=gpurun_out/${1:-r3r4}
shift
M=${@:-resnet18}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2; do
  for m in $M; do
    for tree in _r3base .; do
      tag=$( [ "$tree" = "." ] && echo r4 || echo r3 )
      (cd $tree && timeout -k 10 400 python bench.py --model $m --steps 20 --warmup 5 --comm-figure off) > $O/${m}_${tag}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
      echo "$m $tag rep $r: $(python -c "import json;d=json.load(open('$O/${m}_${tag}_$r.json'));print(d['value'], d['ms_per_step'])")"
    done
  done
done
