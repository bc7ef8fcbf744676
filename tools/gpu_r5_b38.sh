#!/bin/bash
# Round-5 batch 38: stem forward with a kernel row's fragments read ahead of its MFMAs -- A/B of two builds
# of the kernel library (ab/kernels_old.so = previous commit, ab/kernels_new.so = this tree): stem / conv
# GPU tests on the new build, k_stem_fwd kernel-trace time per build (2 runs each), ResNet-18 benches.
set -o pipefail
O=gpurun_out/${1:-r5_b38}
mkdir -p $O
export TMPDIR=/tmp
LIB=pytorch_distributed_example_amd/_lib/_kernels.cpython-310-x86_64-linux-gnu.so
cp ab/kernels_new.so $LIB
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_conv_gpu.py -k stem > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for v in old new; do
    cp ab/kernels_$v.so $LIB
    timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/trace_${v}_$r" -o s \
      -- python3 bench.py --model resnet18 --steps 6 --warmup 2 --comm-figure off > $O/trace_${v}_$r.log 2>&1 || { tail -5 $O/trace_${v}_$r.log; exit 1; }
    python3 - "$O/trace_${v}_$r" $v <<'PY'
import csv, glob, sys
f = glob.glob(f"{sys.argv[1]}/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_stem_fwd" in r["Name"]:
        print(sys.argv[2], "k_stem_fwd avg us", round(float(r["AverageNs"]) / 1e3, 1), "calls", r["Calls"])
PY
  done
done
cp ab/kernels_new.so $LIB
