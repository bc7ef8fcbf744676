#!/bin/bash
# Round-5 batch 39: dgrad requests for the persistent cfg 19 routed to cfg 18 (the transposed-B path gave
# wrong ragged tiles in repeats): the cfg-19 diagnostic, GEMM / transformer GPU tests, GPT-2 benches.
set -o pipefail
O=gpurun_out/${1:-r5_b39}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/gemm_cfg19_check.py > $O/cfg19_check.txt 2>&1 || { tail -20 $O/cfg19_check.txt; exit 1; }
grep -c "mismatches 0 " $O/cfg19_check.txt; grep -v "mismatches 0 " $O/cfg19_check.txt | grep -v amdgpu.ids
timeout -k 10 600 python -u -m pytest -x -q --timeout 170 --timeout-method thread tests/test_gemm_gpu.py tests/test_transformer_gpu.py > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
tail -2 $O/pytest.txt
for r in 1 2; do
  timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 --comm-figure off > $O/gpt2_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  echo "gpt2 rep $r: $(python -c "import json;d=json.load(open('$O/gpt2_$r.json'));print(d['value'], d['ms_per_step'])")"
done
