#!/bin/bash
# In-step phase timeline of the LeNet kernels (tools/lenet_phases.py) on one MI355X.
set -o pipefail
O=gpurun_out/${1:-phases}
mkdir -p $O
timeout -k 10 300 python tools/lenet_phases.py --reps 5 --json $O/phases.json > $O/phases.txt 2>&1
rc=$?
cat $O/phases.txt
exit $rc
