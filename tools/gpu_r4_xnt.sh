#!/bin/bash
# Round-4: non-temporal cross-entropy streaming (PDE_XENT_NT=1) vs default -- xent GPU tests under the
# variant, interleaved GPT-2 benches, per-kernel stats of both (rocprofv3 --stats).
set -o pipefail
O=gpurun_out/${1:-r4_xnt}
mkdir -p $O
export TMPDIR=/tmp
PDE_XENT_NT=1 timeout -k 10 300 python -u -m pytest tests/test_transformer_gpu.py -q -x --timeout 120 --timeout-method thread \
  -k "xent or lm_head or gpt2" > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
tail -1 $O/pytest.txt
bash tools/gpu_gpt2_ab.sh $(basename $O)_ab - "PDE_XENT_NT=1" || exit 1
for v in 0 1; do
  PDE_XENT_NT=$v timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/p$v" -o g -- \
    python3 bench.py --model gpt2 --steps 5 --warmup 2 --comm-figure off > $O/p$v.log 2>&1 || { tail -20 $O/p$v.log; exit 1; }
  rm -f $O/p$v/*kernel_trace.csv
  grep -h "xent" $O/p$v/*kernel_stats.csv | cut -c1-200
done
