#!/bin/bash
# Round-4: split-K reduce with 4 / 8 split loads in flight -- GEMM / transformer GPU tests, same-box GPT-2
# tree A/B against an older worktree ($2), GPT-2 step window.
set -o pipefail
O=gpurun_out/${1:-r4_gred}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_transformer_gpu.py -q --maxfail=10 --timeout 180 \
  --timeout-method thread > $O/pytest.txt 2>&1
TRC=$?
tail -3 $O/pytest.txt
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300
[ $TRC -eq 0 ] || exit $TRC
bash tools/gpu_tree_ab.sh $(basename $O)_ab $2 gpt2 resnet18 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/profg" -o g -- \
  python3 bench.py --model gpt2 --steps 5 --warmup 2 --comm-figure off > $O/profg.log 2>&1 || { tail -20 $O/profg.log; exit 1; }
python3 tools/step_window.py "$(ls $O/profg/*kernel_trace.csv | head -n 1)" k_adamw_master 40 > $O/gpt2_step_window.txt
rm -f $O/profg/*kernel_trace.csv
grep -E "k_gemm_reduce|^step" $O/gpt2_step_window.txt
