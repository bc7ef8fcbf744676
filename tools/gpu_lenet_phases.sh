#!/bin/bash
# Phase stamps of the LeNet step (in-launch optimizer on / off) + driver-config bench on the same box.
set -o pipefail
O=gpurun_out/${1:-lenet_phases}
mkdir -p $O
export TMPDIR=/tmp
for f in defer opt fold; do
  PDE_LENET_BWD_MODE=$f timeout -k 10 120 python tools/lenet_phases.py --reps 5 > $O/phases_$f.txt 2> $O/phases_$f.err || exit 1
  echo "== mode=$f"; grep -v amdgpu.ids $O/phases_$f.txt
  PDE_LENET_BWD_MODE=$f timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/b_$f.json 2> $O/b_$f.err || exit 1
  PDE_LENET_BWD_MODE=$f timeout -k 10 120 python bench.py --steps 2000 --warmup 100 --comm-figure off > $O/bl_$f.json 2> $O/bl_$f.err || exit 1
  python -c "import json;print('bench', json.load(open('$O/b_$f.json'))['ms_per_step'], 'long', json.load(open('$O/bl_$f.json'))['ms_per_step'])"
done
