#!/bin/bash
# Round-5 batch 32: attention.hip built with -fno-slp-vectorize (no packed f32 ops beside the MFMAs) -- A/B of two builds of
# the kernel library (ab/kernels_old.so = previous commit, ab/kernels_new.so = this tree) swapped in
# place: transformer GPU tests on the new build, GPT-2 benches interleaved.
set -o pipefail
O=gpurun_out/${1:-r5_b32}
mkdir -p $O
export TMPDIR=/tmp
LIB=pytorch_distributed_example_amd/_lib/_kernels.cpython-310-x86_64-linux-gnu.so
cp ab/kernels_new.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_transformer_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2 3; do
  for v in old new; do
    cp ab/kernels_$v.so $LIB
    timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 --comm-figure off \
      > $O/gpt2_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "gpt2 $v rep $r: $(python -c "import json;d=json.load(open('$O/gpt2_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
cp ab/kernels_new.so $LIB
