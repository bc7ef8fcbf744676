#!/bin/bash
# Peer tests with cached data regions, then serial-schedule step cost per route (W=1 force_comm).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_peer_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/pytest_peer.log 2>&1; r=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_peer.log | tail -12
[ $r -eq 0 ] || exit $r
B="timeout -k 10 120 python bench.py --steps 2000 --warmup 200 --force-comm"
O=gpurun_out/peer_cached.jsonl
: > $O
PDE_ALLREDUCE_ROUTE=peer1 $B >> $O 2>> gpurun_out/peer_cached.err &&
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1 --nproc-per-node 1 --master-port 29621 tools/peer_bench.py > gpurun_out/peer_bench_w1.json 2> gpurun_out/peer_bench_w1.err
r=$?
python -c "
import json
for l in open('gpurun_out/peer_cached.jsonl'):
    d=json.loads(l); print(d['ms_per_step']*1000, d['config'].get('schedule')); print(json.dumps(d['config'].get('schedule_us_per_step'), indent=0))"
cat gpurun_out/peer_bench_w1.json
exit $r
