#!/bin/bash
# Round-5 batch 5: 256x192 one-shot 8-phase GEMM (cfg 22) tests + timings; non-temporal C stores for the
# LM-head fprop (PDE_GEMM_NT_C_MB) in isolation and in-step.
set -o pipefail
O=gpurun_out/${1:-r5_b5}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 300 --timeout-method thread \
  -k "192_bit_identical or tiles_and_cfgs or gemm8pp" > $O/pytest.txt 2>&1
TRC=$?
if [ $TRC -gt 1 ]; then tail -40 $O/pytest.txt; exit $TRC; fi
grep -E "^(FAILED|ERROR)" $O/pytest.txt | cut -c1-300; tail -2 $O/pytest.txt
timeout -k 10 400 python tools/gemm_own_bench.py --only fprop --cfgs 16,19,22 > $O/gemm.jsonl 2> $O/gemm.err || exit 1
PDE_GEMM_NT_C_MB=256 timeout -k 10 400 python tools/gemm_own_bench.py --only fprop --cfgs 19 > $O/gemm_nt.jsonl 2> $O/gemm_nt.err || exit 1
cat $O/gemm.jsonl $O/gemm_nt.jsonl
bash tools/gpu_gpt2_ab.sh ${1:-r5_b5}/ab - "PDE_LMHEAD_GEMM=own PDE_GEMM_CFG=fprop:50304:768=19 PDE_GEMM_NT_C_MB=256" "PDE_GEMM_FPROP_LIB=none PDE_GEMM_CFG=fprop:768:3072=22,fprop:768:768=16" "PDE_GEMM_CFG=fprop:3072:768=19,dgrad:3072:768=19,fprop:2304:768=22"

# the driver-config window under a kernel trace: per-step GPU time inside the 20-step window
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/prof" -o w -- \
  python3 bench.py --steps 20 --warmup 5 --comm-figure off > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
T=$(ls $O/prof/*kernel_trace.csv | head -n 1)
python3 tools/window_steps.py "$T" 20 6 > $O/window_steps.txt && cat $O/window_steps.txt
rm -f $O/prof/*kernel_trace.csv
exit $TRC
