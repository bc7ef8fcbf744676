#!/bin/bash
# Round-4: deeper in-flight loads in the partial-sum folds (BN finalize / k_fold_rows / LayerNorm
# dgamma-dbeta reduce) -- ResNet / LayerNorm GPU tests, ResNet-18 and GPT-2 benches, both step windows.
set -o pipefail
O=gpurun_out/${1:-r4_fold}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_gpu.py tests/test_transformer_gpu.py -q \
  --maxfail=10 --timeout 180 --timeout-method thread > $O/pytest.txt 2>&1
TRC=$?
tail -3 $O/pytest.txt
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off > $O/rn_$r.json 2>> $O/err.txt &&
  timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 --comm-figure off > $O/gpt2_$r.json 2>> $O/err.txt || exit 1
done
for f in $O/rn_*.json $O/gpt2_*.json; do echo "$(basename $f) $(python3 -c "import json;d=json.load(open('$f'));print(d['value'], d['ms_per_step'])")"; done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window.txt
rm -f $O/prof/*kernel_trace.csv
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/profg" -o g -- \
  python3 bench.py --model gpt2 --steps 5 --warmup 2 --comm-figure off > $O/profg.log 2>&1 || { tail -20 $O/profg.log; exit 1; }
python3 tools/step_window.py "$(ls $O/profg/*kernel_trace.csv | head -n 1)" k_adamw_master 40 > $O/gpt2_step_window.txt
rm -f $O/profg/*kernel_trace.csv
grep -E "fold_rows|finalize|k_ln_reduce|^step" $O/rn_step_window.txt $O/gpt2_step_window.txt
exit $TRC
