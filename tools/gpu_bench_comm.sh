#!/bin/bash
# W=1 headline bench + force-comm bench with full schedule autotuning (incl. fused side-block all-reduce).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python bench.py > gpurun_out/bench_w1.json 2> gpurun_out/bench_w1.err &&
timeout -k 10 200 python bench.py --force-comm > gpurun_out/bench_force_comm.json 2> gpurun_out/bench_force_comm.err
r=$?
python -c "
import json
for f in ('gpurun_out/bench_w1.json', 'gpurun_out/bench_force_comm.json'):
    d=json.load(open(f)); c=d['config']
    print(f, d['ms_per_step']*1000, c['grad_allreduce'], c.get('schedule'))
    if c.get('schedule_us_per_step'): print(json.dumps(c['schedule_us_per_step'], indent=0))"
exit $r
