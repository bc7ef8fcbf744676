#!/bin/bash
# Round-end verification: the full GPU suite, smoke(), the driver-config headline bench and one
# GPT-2 / ResNet-18 bench each.  usage: bash tools/gpu_final.sh <tag>
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/${1:-final}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.txt 2>&1 || { tail -40 $O/pytest_gpu.txt; exit 1; }
tail -2 $O/pytest_gpu.txt
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail -20 $O/smoke.txt; exit 1; }
tail -3 $O/smoke.txt
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver.json 2> $O/bench_driver.err || { tail -20 $O/bench_driver.err; exit 1; }
cut -c1-300 $O/bench_driver.json
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || { tail -20 $O/bench_gpt2.err; exit 1; }
cut -c1-300 $O/bench_gpt2.json
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err || { tail -20 $O/bench_resnet18.err; exit 1; }
cut -c1-300 $O/bench_resnet18.json
