#!/bin/bash
# Round 6: same-box A/B of two builds of BOTH native libraries (ab/{runtime,kernels}_{old,new}.so) on
# the W = 1 comm figure: peer + LeNet GPU tests on the new build, then 5 interleaved 20-step runs and
# 2 interleaved 2000-step runs per arm of bench.py with the comm figure on (headline + w1_rccl_comm).
set -o pipefail
O=gpurun_out/${1:-r6_ab3}
mkdir -p $O
export TMPDIR=/tmp
D=pytorch_distributed_example_amd/_lib
arm() {
  cp ab/runtime_$1.so $D/_runtime.cpython-310-x86_64-linux-gnu.so
  cp ab/kernels_$1.so $D/_kernels.cpython-310-x86_64-linux-gnu.so
}
arm new
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_peer_gpu.py tests/test_lenet_gpu.py > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3 4 5; do
  for v in old new; do
    arm $v
    timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure on > $O/w20_${v}_$r.json 2>> $O/err.txt || exit 1
  done
done
for r in 1 2; do
  for v in old new; do
    arm $v
    timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --comm-figure on > $O/w2000_${v}_$r.json 2>> $O/err.txt || exit 1
  done
done
arm new
python3 - $O <<'PY'
import json, sys, glob, statistics
o = sys.argv[1]
for w in ("w20", "w2000"):
    for v in ("old", "new"):
        rows = [json.load(open(f)) for f in sorted(glob.glob(f"{o}/{w}_{v}_*.json"))]
        h = [d["ms_per_step"] * 1000 for d in rows]
        c = [d["w1_rccl_comm"]["ms_per_step"] * 1000 for d in rows]
        dc = [b - a for a, b in zip(h, c)]
        print(w, v, "headline", [round(x, 2) for x in h], "comm", [round(x, 2) for x in c],
              "comm-headline", [round(x, 2) for x in dc], "median", round(statistics.median(dc), 2))
PY
