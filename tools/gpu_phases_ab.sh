#!/bin/bash
# In-step phase stamps: round-2 baseline worktree vs the current tree, same box.
set -o pipefail
O=gpurun_out/${1:-phases_ab}
mkdir -p $O
for v in base new; do
  if [ $v = base ]; then D=_r2base; else D=.; fi
  (cd $D && timeout -k 10 120 python tools/lenet_phases.py --reps 7) > $O/$v.txt 2> $O/$v.err || exit 1
  echo "== $v"; grep -v amdgpu.ids $O/$v.txt | python -c "
import sys, json
for l in sys.stdin:
    k, j = l.split(' ', 1); d = json.loads(j)
    r = {x: d[x] for x in ('start', 'end', 'block_dur_p50', 'block_dur_max')}
    if 'roles' in d: r['roles'] = {n: (v['end_max'], v['phases_p50']) for n, v in d['roles'].items()}
    if 'dur_by_block_range' in d: r['ranges'] = list(d['dur_by_block_range'].values())
    print(k, json.dumps(r))"
done
