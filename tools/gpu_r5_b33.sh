#!/bin/bash
# Round-5 batch 33: lenet_v2.hip built with -fno-slp-vectorize -- A/B of two builds of the kernel
# library (ab/kernels_old.so = previous commit, ab/kernels_new.so = this tree) swapped in place:
# toy-CNN GPU tests on the new build, driver-config headline benches interleaved.
set -o pipefail
O=gpurun_out/${1:-r5_b33}
mkdir -p $O
export TMPDIR=/tmp
LIB=pytorch_distributed_example_amd/_lib/_kernels.cpython-310-x86_64-linux-gnu.so
cp ab/kernels_new.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_lenet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2 3 4; do
  for v in old new; do
    cp ab/kernels_$v.so $LIB
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/b_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/long_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "$v rep $r: $(python -c "import json;d=json.load(open('$O/b_${v}_$r.json'));e=json.load(open('$O/long_${v}_$r.json'));print(d['value'], d['ms_per_step']*1e3, '| 2000 steps', e['ms_per_step']*1e3)")"
  done
done
cp ab/kernels_new.so $LIB
