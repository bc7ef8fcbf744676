#!/bin/bash
# Round-4: ResNet-18 BN-backward reduction fused into conv2's dgrad epilogue -- conv / ResNet GPU tests,
# interleaved same-box benches (PDE_RESNET_BNB_FUSE=1 default vs 0), then the W=1 step window of both.
set -o pipefail
O=gpurun_out/${1:-r4_bnb}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_resnet_gpu.py -q --maxfail=10 --timeout 180 \
  --timeout-method thread > $O/pytest.txt 2>&1
TRC=$?
tail -3 $O/pytest.txt
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300
for r in 1 2; do
  timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off > $O/A_$r.json 2>> $O/err.txt &&
  PDE_RESNET_BNB_FUSE=0 timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off \
    > $O/B_$r.json 2>> $O/err.txt || exit 1
done
for f in $O/A_*.json $O/B_*.json; do echo "$(basename $f) $(python3 -c "import json;d=json.load(open('$f'));print(d['value'], d['ms_per_step'])")"; done
timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/prof" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
python3 tools/step_window.py "$(ls $O/prof/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window.txt
rm -f $O/prof/*kernel_trace.csv
PDE_RESNET_BNB_FUSE=0 timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/profB" -o rn -- \
  python3 bench.py --model resnet18 --steps 5 --warmup 2 --comm-figure off > $O/profB.log 2>&1 || { tail -20 $O/profB.log; exit 1; }
python3 tools/step_window.py "$(ls $O/profB/*kernel_trace.csv | head -n 1)" k_sgd_master 45 > $O/rn_step_window_nofuse.txt
rm -f $O/profB/*kernel_trace.csv
head -12 $O/rn_step_window.txt
head -12 $O/rn_step_window_nofuse.txt
exit $TRC
