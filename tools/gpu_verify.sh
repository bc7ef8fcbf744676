#!/bin/bash
# Round verification on one MI355X (gpurun): driver-style bench, long bench, GPU tests.
set -o pipefail
O=gpurun_out/${1:-verify}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 300 python bench.py --gpus 1 --steps 2000 --warmup 200 --comm-figure off > $O/bench_long.json 2> $O/bench_long.err &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1
rc=$?
tail -3 $O/pytest_gpu.txt
cat $O/bench_driver.json $O/bench_long.json
exit $rc
