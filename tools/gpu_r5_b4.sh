#!/bin/bash
# Round-5 batch 4: continuous GEMM (cfgs 20 / 21) after hoisting the tile-origin divisions; peer fixes.
set -o pipefail
O=gpurun_out/${1:-r5_b4}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
  -k "gemm8pc or schedules_match or peer_inplace" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
timeout -k 10 300 python tools/gemm_own_bench.py --only fprop,dgrad --cfgs 16,19,20,21 > $O/gemm.jsonl 2> $O/gemm.err || exit 1
cat $O/gemm.jsonl
exit $TRC
