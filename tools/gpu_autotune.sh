#!/bin/bash
# Peer / autotune tests, then force-comm benches (W=1) with whole-step schedule autotuning.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_peer_gpu.py -v --timeout 150 --timeout-method thread > gpurun_out/pytest_peer.log 2>&1; r=$?
grep -E "PASS|FAIL|passed|failed" gpurun_out/pytest_peer.log | tail -12
[ $r -eq 0 ] || exit $r
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --force-comm > gpurun_out/bench_force_comm.json 2> gpurun_out/bench_force_comm.err &&
python -c "
import json; d=json.load(open('gpurun_out/bench_force_comm.json')); c=d['config']
print(d['ms_per_step']*1000, c['grad_allreduce'], c.get('schedule')); print(json.dumps(c.get('schedule_us_per_step'), indent=0))"
