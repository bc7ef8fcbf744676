#!/bin/bash
# xGMI peer all-reduce on one GPU (ranks share cuda:0), then the engine W=1 comm tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_peer_gpu.py -v -x --timeout 150 --timeout-method thread > gpurun_out/pytest_peer.log 2>&1; r=$?
tail -15 gpurun_out/pytest_peer.log
[ $r -eq 0 ] || exit $r
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -v -k "engine_comm or ddp or collectives" --timeout 150 --timeout-method thread > gpurun_out/pytest_peer2.log 2>&1; r=$?
tail -8 gpurun_out/pytest_peer2.log
exit $r
