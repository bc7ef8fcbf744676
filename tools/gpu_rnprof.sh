#!/bin/bash
# ResNet-18 kernel profile (rocprofv3 --kernel-trace --stats) of a short bench run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_rn" -o rn \
  -- python3 bench.py --model resnet18 --steps 4 --warmup 3 > gpurun_out/prof_rn.log 2>&1
r=$?
tail -3 gpurun_out/prof_rn.log
exit $r
