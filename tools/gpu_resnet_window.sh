#!/bin/bash
# Round-4: ResNet-18 W=1 step-window kernel trace (graph mode) -> per-kernel breakdown of one step.
set -o pipefail
O=gpurun_out/${1:-r4_rnprof}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window.txt
rm -f $O/prof/*kernel_trace.csv
head -45 $O/rn_step_window.txt
