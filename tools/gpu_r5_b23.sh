#!/bin/bash
# Round-5 batch 23: fused BN + ReLU + max-pool forward variants incl. 512-thread vertical pairs:
# variant test, micro-timings, ResNet-18 bench A/B (PDE_BNPOOL_FWD=1 vs 3), interleaved.
set -o pipefail
O=gpurun_out/${1:-r5_b23}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_resnet_gpu.py \
  -k "maxpool" > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
timeout -k 10 200 python tools/bnpool_bench.py --rounds 5 > $O/bnpool.jsonl 2> $O/bnpool.err || { tail -20 $O/bnpool.err; exit 1; }
cat $O/bnpool.jsonl
for r in 1 2 3; do
  for v in 1 2 3; do
    PDE_BNPOOL_FWD=$v timeout -k 10 400 python bench.py --model resnet18 --steps 30 --warmup 5 --comm-figure off \
      > $O/rn_${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
    echo "variant $v rep $r: $(python -c "import json;d=json.load(open('$O/rn_${v}_$r.json'));print(d['value'], d['ms_per_step'])")"
  done
done
