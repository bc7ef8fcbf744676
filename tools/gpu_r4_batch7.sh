#!/bin/bash
# Round-4 batch 7: GPT-2 with the cfg-18 GEMM table + the own LM-head dgrad (default) against the
# round-4 table (same box, interleaved), then instruction-fetch PMC passes over the headline step.
set -o pipefail
O=gpurun_out/${1:-r4_b7}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_transformer_gpu.py -q -x --timeout 120 --timeout-method thread -k "gpt2 or lm_head or xent" > $O/pytest.txt 2>&1
TRC=$?; tail -2 $O/pytest.txt; [ $TRC -eq 0 ] || exit $TRC
bash tools/gpu_gpt2_ab.sh $(basename $O)_ab - "PDE_LMHEAD_GEMM=lib PDE_GEMM_CFG=wgrad:3072:768=9/5,wgrad:768:3072=9/5,wgrad:2304:768=9/7,wgrad:50304:768=11/2,dgrad:3072:768=15,dgrad:768:50304=9" || exit 1
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_IFETCH SQ_INSTS_VALU" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/pmc$i" -o pmc --pmc $grp \
      -- python3 bench.py --steps 100 --warmup 10 --comm-figure off > $O/pmc$i.log 2>&1 || { echo "pmc group $i failed"; tail -5 $O/pmc$i.log; }
done
python3 tools/pmc_summary.py $(ls $O/pmc*/*counter_collection.csv) > $O/pmc_summary.md 2>&1 || true
head -30 $O/pmc_summary.md
