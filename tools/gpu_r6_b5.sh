#!/bin/bash
# Round 6 batch 5: step-window kernel traces of the final build (GPT-2 and ResNet-18, W=1, graph replay),
# and the toy-CNN 20-step window anatomy (host vs GPU time of the window, PDE_BENCH_TRACE).
set -o pipefail
O=gpurun_out/${1:-r6_b5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/gp" -o gp -- \
  python3 bench.py --model gpt2 --steps 5 --warmup 2 --comm-figure off > $O/gp.log 2>&1 || { tail -20 $O/gp.log; exit 1; }
python3 tools/step_window.py "$(ls $O/gp/*kernel_trace.csv | head -n 1)" k_adamw_master 40 > $O/gpt2_step_window.txt || exit 1
rm -f $O/gp/*kernel_trace.csv
timeout -k 10 500 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/rn" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/rn.log 2>&1 || { tail -20 $O/rn.log; exit 1; }
python3 tools/step_window.py "$(ls $O/rn/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window.txt || exit 1
rm -f $O/rn/*kernel_trace.csv
for i in 1 2 3; do
  PDE_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/w20_$i.json 2> $O/w20_$i.err || exit 1
  PDE_BENCH_TRACE=1 timeout -k 10 300 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/w2000_$i.json 2> $O/w2000_$i.err || exit 1
done
head -30 $O/gpt2_step_window.txt; head -30 $O/rn_step_window.txt
for f in $O/w20_*.err $O/w2000_*.err; do echo "$f $(grep trace_ $f)"; done
