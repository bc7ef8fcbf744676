#!/bin/bash
# Round-4 batch 5: DDP graph capture over the RCCL routes (watchdog thread now in relaxed capture
# mode), the LM-head scale kernel, GPT-2 parity; then the GPT-2 bench (W=1 comm figure), the headline
# bench, and a GPT-2 step-window kernel trace.
set -o pipefail
O=gpurun_out/${1:-r4_b5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_peer_gpu.py tests/test_transformer_gpu.py -q --maxfail=10 --timeout 180 \
  --timeout-method thread -k "ddp_graph or scale_bf16 or gpt2 or xent or lm_head" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
timeout -k 10 400 python3 bench.py --model gpt2 > $O/gpt2.json 2> $O/gpt2.err || { tail -20 $O/gpt2.err; exit 1; }
cut -c1-400 $O/gpt2.json
timeout -k 10 300 python3 bench.py > $O/lenet.json 2> $O/lenet.err || { tail -20 $O/lenet.err; exit 1; }
cut -c1-1200 $O/lenet.json
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof_gpt2" -o gpt2 -- \
  python3 bench.py --model gpt2 --steps 5 --warmup 2 --comm-figure off > $O/prof_gpt2.log 2>&1 || { tail -20 $O/prof_gpt2.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof_gpt2/*kernel_trace.csv | head -n 1)" k_adamw_master 40 > $O/gpt2_step_window.txt
rm -f $O/prof_gpt2/*kernel_trace.csv
head -30 $O/gpt2_step_window.txt
exit $TRC
