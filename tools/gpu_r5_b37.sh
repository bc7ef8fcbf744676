#!/bin/bash
# Round-5 batch 37: k_hconv and k_igemm epilogue statistics only when requested (k_hconv: row mask only
# on partial fragments) -- A/B of two builds of the kernel library
# (ab/kernels_old.so = previous commit, ab/kernels_new.so = this tree), swapped in place between runs:
# conv / ResNet GPU tests on the new build, per-layer conv timings and ResNet-18 benches, interleaved.
set -o pipefail
O=gpurun_out/${1:-r5_b37}
mkdir -p $O
export TMPDIR=/tmp
LIB=pytorch_distributed_example_amd/_lib/_kernels.cpython-310-x86_64-linux-gnu.so
cp ab/kernels_new.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py \
  tests/test_resnet_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for v in old new; do
    cp ab/kernels_$v.so $LIB
    timeout -k 10 300 python tools/conv_bench.py --stages 2 > $O/conv_${v}_$r.jsonl 2> $O/conv.err || { tail -20 $O/conv.err; exit 1; }
    python - $O/conv_${v}_$r.jsonl $v <<'PY'
import json, sys
out, tot = [], 0.0
for l in open(sys.argv[1]):
    d = json.loads(l)
    if "fprop_us" in d:
        out.append(f'{d["layer"]} {d["fprop_us"]}/{d["dgrad_us"]}/{d["wgrad_us"]}')
        tot += (d["fprop_us"] + d["dgrad_us"] + d["wgrad_us"]) * d["count"]
print(sys.argv[2], "conv total", round(tot, 1), " ".join(out))
PY
  done
done
for r in 1 2 3; do
  for v in old new; do
    cp ab/kernels_$v.so $LIB
    timeout -k 10 400 python bench.py --model resnet18 --steps 30 --warmup 5 --comm-figure off \
      > $O/rn_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "$v rep $r: $(python -c "import json;d=json.load(open('$O/rn_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
cp ab/kernels_new.so $LIB
