#!/bin/bash
# Round-4 batch 4: DDP graph-capture tests over the RCCL routes + the peer route, then a rocprofv3
# kernel-trace of the headline step (per-kernel stats) and of one GPT-2 step window.
set -o pipefail
O=gpurun_out/${1:-r4_b4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_peer_gpu.py -q --maxfail=10 --timeout 180 --timeout-method thread -k "ddp_graph" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_lenet" -o lenet -- \
  python3 bench.py --steps 200 --warmup 20 --comm-figure off > $O/prof_lenet.log 2>&1 || { tail -20 $O/prof_lenet.log; exit 1; }
python3 tools/prof_summary.py "$(ls $O/prof_lenet/*kernel_stats.csv | head -n 1)" > $O/lenet_kernel_stats.md 2>&1 || true
rm -f $O/prof_lenet/*kernel_trace.csv
head -20 $O/lenet_kernel_stats.md
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_gpt2" -o gpt2 -- \
  python3 bench.py --model gpt2 --steps 5 --warmup 2 --comm-figure off > $O/prof_gpt2.log 2>&1 || { tail -20 $O/prof_gpt2.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof_gpt2/*kernel_trace.csv | head -n 1)" k_adamw_master 40 > $O/gpt2_step_window.txt
rm -f $O/prof_gpt2/*kernel_trace.csv
head -30 $O/gpt2_step_window.txt
exit $TRC
