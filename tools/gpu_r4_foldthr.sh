#!/bin/bash
# Round-4: BN partial-row fold threshold (PDE_BN_FOLD_THRESHOLD: 256 default / 512 / 2048) -- ResNet GPU
# tests at 2048, interleaved ResNet-18 benches of the three settings, step window at the best candidate.
set -o pipefail
O=gpurun_out/${1:-r4_foldthr}
mkdir -p $O
export TMPDIR=/tmp
PDE_BN_FOLD_THRESHOLD=2048 timeout -k 10 600 python -u -m pytest tests/test_resnet_gpu.py tests/test_conv_gpu.py -q -x \
  --timeout 180 --timeout-method thread > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2; do
  for t in 256 512 2048; do
    PDE_BN_FOLD_THRESHOLD=$t timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off \
      > $O/t${t}_$r.json 2>> $O/err.txt || exit 1
    echo "thr $t rep $r: $(python3 -c "import json;d=json.load(open('$O/t${t}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
for t in 512 2048; do
  PDE_BN_FOLD_THRESHOLD=$t timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/p$t" -o rn -- \
    python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/p$t.log 2>&1 || { tail -20 $O/p$t.log; exit 1; }
  python3 tools/step_window.py "$(ls $O/p$t/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window_t$t.txt
  rm -f $O/p$t/*kernel_trace.csv
  grep -E "^step|fold_rows|finalize" $O/rn_step_window_t$t.txt
done
