#!/bin/bash
# LeNet GPU tests, then the interleaved A/B against the round-2 baseline worktree.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_lenet_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lenet.txt 2>&1; rc=$?; tail -4 gpurun_out/pytest_lenet.txt; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_ab.sh ${1:-ab} $2
