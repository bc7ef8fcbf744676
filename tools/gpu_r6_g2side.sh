#!/bin/bash
# Round 6: split-K wgrad reductions on a side stream (PDE_WGRAD_SIDE): the GPU test, then GPT-2 benches
# with the switch off / on, interleaved.
set -o pipefail
O=gpurun_out/${1:-r6_g2side}; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 150 --timeout-method thread tests/test_transformer_gpu.py -k "side_stream or step_replays or trains" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
for r in 1 2 3; do
  for v in 0 1; do
    PDE_WGRAD_SIDE=$v timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 --comm-figure off > $O/g2_side${v}_$r.json 2>> $O/err.txt || exit 1
    python3 -c "import json;d=json.load(open('$O/g2_side${v}_$r.json'));print('side $v',$r,d['value'],d['ms_per_step'])"
  done
done
