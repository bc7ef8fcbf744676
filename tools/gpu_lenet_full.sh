#!/bin/bash
# LeNet numerics / determinism / comm-schedule GPU tests.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_lenet_gpu.py tests/test_ops_gpu.py tests/test_peer_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_lenet_full.txt 2>&1; rc=$?; tail -4 gpurun_out/pytest_lenet_full.txt; exit $rc
