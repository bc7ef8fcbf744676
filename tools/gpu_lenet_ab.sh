#!/bin/bash
# LeNet engine tests + A/B bench of an engine switch (env var given as $1, default PDE_LENET_FUSE_HEAD).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
VAR=${1:-PDE_LENET_FUSE_HEAD}
timeout -k 10 400 python -u -m pytest tests/test_lenet_gpu.py tests/test_ops_gpu.py -q --timeout 150 --timeout-method thread -x > gpurun_out/pytest_lenet.log 2>&1; r=$?
tail -2 gpurun_out/pytest_lenet.log
[ $r -eq 0 ] || exit $r
: > gpurun_out/lenet_ab.txt
for rep in 1 2 3; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 120 python bench.py --steps 3000 --warmup 300 > gpurun_out/ab.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/ab.json')); print('$VAR=$v', d['ms_per_step']*1000)" >> gpurun_out/lenet_ab.txt
  done
done
cat gpurun_out/lenet_ab.txt
