#!/bin/bash
# Iteration loop on one MI355X: targeted GPU tests, in-step phase timeline, short + long bench.
# usage: bash tools/gpu_iter.sh <tag> [pytest -k expression]
set -o pipefail
O=gpurun_out/${1:-iter}
K=${2:-lenet}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "$K" > $O/pytest.txt 2>&1 &&
timeout -k 10 200 python tools/lenet_phases.py --reps 5 --json $O/phases.json > $O/phases.txt 2>&1 &&
timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/bench20.json 2> $O/bench20.err &&
timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/bench2000.json 2> $O/bench2000.err
rc=$?
tail -5 $O/pytest.txt; cat $O/phases.txt $O/bench20.json $O/bench2000.json 2>/dev/null | cut -c1-600
exit $rc
