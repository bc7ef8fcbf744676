#!/bin/bash
# Round-4: one BN partial row per persistent k_hconv64 block (no k_fold_rows for layer 1) -- conv /
# ResNet GPU tests, then a same-box tree A/B against the previous commit's worktree ($2) and the step window.
set -o pipefail
O=gpurun_out/${1:-r4_rows}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_gpu.py -q --maxfail=10 --timeout 180 \
  --timeout-method thread > $O/pytest.txt 2>&1
TRC=$?
tail -3 $O/pytest.txt
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300
[ $TRC -eq 0 ] || exit $TRC
bash tools/gpu_tree_ab.sh $(basename $O)_ab $2 resnet18 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window.txt
rm -f $O/prof/*kernel_trace.csv
head -20 $O/rn_step_window.txt
