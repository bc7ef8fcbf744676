#!/bin/bash
# ResNet-18 iteration: ResNet / conv GPU tests, the ResNet-18 bench (x2) and its step window under rocprofv3.
# usage: bash tools/gpu_rn.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-rn}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_resnet_gpu.py -x -q --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_rn_$r.json 2> $O/bench_rn_$r.err || { tail -20 $O/bench_rn_$r.err; exit 1; }
  cut -c1-200 $O/bench_rn_$r.json
done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof/*kernel_trace.csv | head -n 1)" k_sgd_master 60 > $O/rn_step_window.txt
rm -f $O/prof/*kernel_trace.csv
head -30 $O/rn_step_window.txt
