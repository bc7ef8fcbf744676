#!/bin/bash
# Round-4 batch: ResNet head / parity / DDP-graph tests, LeNet phases per conv-gradient reduction mode,
# GPT-2 LM-head variants A/B.
set -o pipefail
O=gpurun_out/${1:-r4_b2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 180 --timeout-method thread -k "resnet_head or gpu_matches_cpu or catches_broken or ddp_graph" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-400; tail -2 $O/pytest.txt
for m in defer ext fold; do
  PDE_LENET_BWD_MODE=$m timeout -k 10 200 python tools/lenet_phases.py --reps 5 > $O/phases_$m.txt 2>&1 || exit 1
  echo "== $m"; grep -h "^conv_bwd\|^adam" $O/phases_$m.txt | cut -c1-120
done
bash tools/gpu_gpt2_ab.sh ${1:-r4_b2}/gpt2 - PDE_LMHEAD_CHUNK=2048 PDE_LMHEAD_GEMM=lib "PDE_LMHEAD_CHUNK=2048 PDE_LMHEAD_GEMM=lib"
exit $TRC
