#!/bin/bash
# Round-3 iteration 2: window-probe variants, DDP peer route + ops/transformer/resnet GPU tests,
# GPT-2 and ResNet benches.
set -o pipefail
O=gpurun_out/${1:-iter2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/window_probe2.py > $O/wp2.json 2> $O/wp2.err || exit 1
cat $O/wp2.json
timeout -k 10 900 python -u -m pytest tests/test_peer_gpu.py tests/test_ops_gpu.py tests/test_transformer_gpu.py tests/test_resnet_gpu.py tests/test_conv_gpu.py -x -q --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1; rc=$?; tail -4 $O/pytest.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model gpt2 --steps 20 --warmup 5 > $O/bench_gpt2.json 2> $O/bench_gpt2.err || exit 1
timeout -k 10 300 python bench.py --model resnet18 --steps 20 --warmup 5 > $O/bench_resnet18.json 2> $O/bench_resnet18.err || exit 1
python -c "import json;[print(k, json.load(open('$O/bench_'+k+'.json'))['value']) for k in ('gpt2','resnet18')]"
