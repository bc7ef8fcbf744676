#!/bin/bash
# Kernel timeline of one training step with the peer all-reduce in the overlapped schedule (W=1 force_comm).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for route in peer1 rccl; do
  PDE_ALLREDUCE_ROUTE=$route timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d "$PWD/gpurun_out/tr_$route" -o tr \
    -- python3 bench.py --steps 200 --warmup 20 --force-comm --no-autotune > gpurun_out/tr_$route.log 2>&1 || exit $?
  f=$(find gpurun_out/tr_$route -name "*kernel_trace.csv" | head -1)
  echo "== $route"; python3 tools/trace_summary.py "$f" k_conv_fwd 14
done
