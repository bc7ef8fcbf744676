#!/bin/bash
# One PMC pass of instruction-mix counters over the ResNet-18 bench (eager), per-kernel means for the
# convolution kernels.  usage: bash tools/gpu_pmc_valu.sh <tag>
set -o pipefail
O=gpurun_out/${1:-pmc_valu}
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d "$PWD/$O/g1" -o rn \
    --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES \
    -- python3 bench.py --model resnet18 --steps 2 --warmup 1 --model-graph off > $O/g1.log 2>&1 || { tail -5 $O/g1.log; exit 1; }
python3 tools/pmc_pick.py $O k_hwgrad64 k_hconv64 "k_hconv<128" "k_wgrad<128" "k_wgrad<64" "k_igemm<128" "k_igemm<256"
