#!/bin/bash
# Round-3 start: new peer self-test (stale injection), driver-style benches of the three configs.
set -o pipefail
O=gpurun_out/${1:-r3_start}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_peer_gpu.py -x -v --timeout 200 --timeout-method thread > $O/pytest_peer.txt 2>&1 &&
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err &&
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err &&
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err
rc=$?
tail -3 $O/pytest_peer.txt
cat $O/bench_driver.json $O/bench_gpt2.json $O/bench_resnet18.json
exit $rc
