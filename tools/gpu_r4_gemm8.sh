#!/bin/bash
# Round-4: the 8-phase GEMM (cfg 18) -- GEMM tests, isolated timings of every GPT-2 GEMM against the
# 2-phase configs, then the GPT-2 step with the GEMMs moved to cfg 18 (same-box A/B).
set -o pipefail
O=gpurun_out/${1:-r4_gemm8}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py -q -x --timeout 120 --timeout-method thread > $O/pytest.txt 2>&1
TRC=$?
tail -3 $O/pytest.txt
if [ $TRC -ne 0 ]; then grep -E "^(FAILED|ERROR)|Error" $O/pytest.txt | head -20; exit $TRC; fi
timeout -k 10 500 python tools/gemm_own_bench.py --cfgs ${GCFGS:-9,15,16,17,18} --out $O/gemm.jsonl > $O/gemm.log 2>&1 || { tail -20 $O/gemm.log; exit 1; }
python3 - $O/gemm.jsonl <<'PY'
import json, sys
for ln in open(sys.argv[1]):
    d = json.loads(ln)
    own = d["own_us"]
    keep = {k: v for k, v in own.items() if str(k).split("/")[0] in ("9", "15", "16", "17", "18")}
    b18 = min((v for k, v in own.items() if str(k).split("/")[0] == "18"), default=None)
    print(d["gemm"], "lib", d["lib_us"], "best", d["best"], own[str(d["best"])] if str(d["best"]) in own else own.get(d["best"]), "cfg18", b18)
PY
[ -n "$NOAB" ] || bash tools/gpu_gpt2_ab.sh ${1:-r4_gemm8}_ab - "PDE_GEMM_CFG=fprop:2304:768=18,fprop:3072:768=18" "PDE_GEMM_CFG=fprop:2304:768=18,fprop:3072:768=18,dgrad:768:2304=18,dgrad:768:768=18,dgrad:768:3072=18,dgrad:3072:768=18,wgrad:2304:768=18/9,wgrad:768:768=18/26,wgrad:3072:768=18/7,wgrad:768:3072=18/7"
