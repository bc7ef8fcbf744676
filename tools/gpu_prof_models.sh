#!/bin/bash
# rocprofv3 kernel stats of the GPT-2 and ResNet-18 benches (5 timed + 2 warm-up steps each) and markdown
# summaries under gpurun_out/<tag>/.  usage: bash tools/gpu_prof_models.sh <tag> [rn|gpt|all]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-prof_models}
WHICH=${2:-all}
mkdir -p $O
export TMPDIR=/tmp
prof() {   # $1 = model name, $2 = short tag
  timeout -k 10 500 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$O/$2" -o $2 -- \
    python3 bench.py --model $1 --steps 5 --warmup 2 > $O/$2.log 2>&1 &&
  python3 tools/prof_summary.py "$(ls $O/$2/*kernel_stats.csv | head -n 1)" "$1 (bench --steps 5 --warmup 2)" 7 > $O/$2_stats.md
}
rc=0
if [ "$WHICH" = rn ] || [ "$WHICH" = all ]; then prof resnet18 rn || rc=$?; fi
if [ $rc = 0 ] && { [ "$WHICH" = gpt ] || [ "$WHICH" = all ]; }; then prof gpt2 gpt2 || rc=$?; fi
head -n 40 $O/*_stats.md
exit $rc
