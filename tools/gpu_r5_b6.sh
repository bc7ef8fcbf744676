#!/bin/bash
# Round-5 batch 6: GPT-2 on the framework's GEMMs only (no hipBLASLt): GEMM + transformer GPU tests,
# fprop timings of the 256x192 8-phase loop, GPT-2 bench x2, and the step window kernel list.
set -o pipefail
O=gpurun_out/${1:-r5_b6}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gemm_gpu.py tests/test_transformer_gpu.py -m gpu -q --maxfail=10 \
  --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
timeout -k 10 400 python tools/gemm_own_bench.py --only fprop --cfgs 16,22 > $O/gemm.jsonl 2> $O/gemm.err || exit 1
cat $O/gemm.jsonl
for r in 1 2; do
  timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_$r.json 2>> $O/err.txt || exit 1
  echo "gpt2 rep $r: $(python -c "import json;d=json.load(open('$O/gpt2_$r.json'));print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/prof" -o g -- \
  python3 bench.py --model gpt2 --steps 6 --warmup 2 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
T=$(ls $O/prof/*kernel_trace.csv | head -n 1)
python3 tools/step_window.py "$T" k_adamw_master 40 > $O/gpt2_step_window.txt && cat $O/gpt2_step_window.txt
rm -f $O/prof/*kernel_trace.csv
exit $TRC
