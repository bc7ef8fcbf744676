#!/bin/bash
# All-reduce route timings (W=1 real RCCL vs peer; W=2/4 ranks sharing cuda:0) + multi-rank bench rehearsal.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
RUN="python -m torch.distributed.run --nnodes=1 --master-addr 127.0.0.1"
timeout -k 10 120 $RUN --nproc-per-node 1 --master-port 29611 tools/peer_bench.py > gpurun_out/peer_bench_w1.json 2> gpurun_out/peer_bench_w1.err && cat gpurun_out/peer_bench_w1.json &&
timeout -k 10 120 $RUN --nproc-per-node 2 --master-port 29612 tools/peer_bench.py --shared-gpu > gpurun_out/peer_bench_w2s.json 2> gpurun_out/peer_bench_w2s.err && cat gpurun_out/peer_bench_w2s.json &&
timeout -k 10 120 $RUN --nproc-per-node 4 --master-port 29613 tools/peer_bench.py --shared-gpu > gpurun_out/peer_bench_w4s.json 2> gpurun_out/peer_bench_w4s.err && cat gpurun_out/peer_bench_w4s.json &&
timeout -k 10 200 $RUN --nproc-per-node 2 --master-port 29614 bench.py --gpus 2 --shared-gpu --steps 500 --warmup 50 > gpurun_out/bench_w2_shared.json 2> gpurun_out/bench_w2_shared.err && cat gpurun_out/bench_w2_shared.json &&
timeout -k 10 200 $RUN --nproc-per-node 1 --master-port 29615 bench.py --gpus 1 > gpurun_out/bench_w1_torchrun.json 2> gpurun_out/bench_w1_torchrun.err && cat gpurun_out/bench_w1_torchrun.json
rc=$?
echo "rc=$rc"
exit $rc
