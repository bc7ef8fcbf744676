#!/bin/bash
# Round-5 batch 15: conv weight gradients on a side stream (utils/sidestream.py): ResNet GPU tests,
# DDP graph / peer tests, then same-box interleaved ResNet-18 benches with the side stream on / off.
set -o pipefail
O=gpurun_out/${1:-r5_b15}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_resnet_gpu.py \
  tests/test_peer_gpu.py -k "resnet or ddp" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  for v in 1 0; do
    PDE_WGRAD_STREAM=$v timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 --comm-figure off \
      > $O/rn_s${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "side=$v rep $r: $(python -c "import json;d=json.load(open('$O/rn_s${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
