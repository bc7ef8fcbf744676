#!/bin/bash
# Round-4: staggered 8-phase GEMM -- tests, isolated timings (cfgs 16/17/18), then PMC passes of the
# c_fc weight gradient (3072 x 768 x 16384, 7 splits) on cfg 18 and cfg 17.
set -o pipefail
O=gpurun_out/${1:-r4_gemm8b}
mkdir -p $O
export TMPDIR=/tmp
GCFGS=16,17,18 NOAB=1 bash tools/gpu_r4_gemm8.sh $(basename $O) || exit $?
for c in 18 17; do
  GEMM_ARGS="--kind wgrad --M 3072 --N 768 --K 16384 --cfg $c --splits 7 --reps 10" bash tools/gpu_gemm_pmc.sh wgrad_cfg$c > $O/pmc_$c.log 2>&1 || { tail -5 $O/pmc_$c.log; exit 1; }
done
mkdir -p $O/pmc && for c in 18 17; do for g in 1 2 3; do cp $(ls gpurun_out/gemm_pmc/wgrad_cfg$c/g$g/*counter_collection.csv | head -n 1) $O/pmc/cfg${c}_g$g.csv; done; done
rm -rf gpurun_out/gemm_pmc
echo pmc-done
