#!/bin/bash
# In-step cost of the W>1 communication path measured at W=1 (force_comm): RCCL vs peer routes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="timeout -k 10 120 python bench.py --steps 2000 --warmup 200"
O=gpurun_out/comm_overhead.jsonl
: > $O
$B >> $O 2>> gpurun_out/comm_overhead.err &&
$B --force-comm >> $O 2>> gpurun_out/comm_overhead.err &&
PDE_ALLREDUCE_ROUTE=peer1 $B --force-comm >> $O 2>> gpurun_out/comm_overhead.err &&
PDE_ALLREDUCE_ROUTE=peer2 $B --force-comm >> $O 2>> gpurun_out/comm_overhead.err &&
PDE_ALLREDUCE_ROUTE=peer1 $B --force-comm --no-overlap >> $O 2>> gpurun_out/comm_overhead.err &&
PDE_ALLREDUCE_ROUTE=rccl $B --force-comm --no-overlap >> $O 2>> gpurun_out/comm_overhead.err
r=$?
python - <<'PY'
import json
for l in open("gpurun_out/comm_overhead.jsonl"):
    d = json.loads(l); c = d["config"]
    print(d["ms_per_step"] * 1000, c["grad_allreduce"], c.get("routes"), d["comm_errors"])
PY
exit $r
