#!/bin/bash
# Round-4 batch 3: ResNet parity / DDP-graph tests, GPT-2 LM-head GEMM routes, model benches with the
# W=1 communication figure (DDP collectives captured in the step graph).
set -o pipefail
O=gpurun_out/${1:-r4_b3}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 180 --timeout-method thread -k "resnet_head or gpu_matches_cpu or catches_broken or ddp_graph" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-400; tail -2 $O/pytest.txt
bash tools/gpu_gpt2_ab.sh ${1:-r4_b3}/gpt2 - PDE_LMHEAD_GEMM=own PDE_LMHEAD_GEMM=lib3 || exit 1
timeout -k 10 400 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/gpt2_comm.json 2> $O/gpt2_comm.err || { tail -20 $O/gpt2_comm.err; exit 1; }
timeout -k 10 400 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/rn_comm.json 2> $O/rn_comm.err || { tail -20 $O/rn_comm.err; exit 1; }
python - $O <<'PY'
import json, sys
o = sys.argv[1]
for f in ("gpt2_comm.json", "rn_comm.json"):
    d = json.load(open(f"{o}/{f}"))
    w = d.get("w1_rccl_comm", {})
    print(f, d["value"], d["ms_per_step"], "| comm:", w.get("value"), w.get("ms_per_step"), w.get("mode"), w.get("grad_reduce_route"), w.get("bucket_mb"), w.get("error"))
PY
exit $TRC
