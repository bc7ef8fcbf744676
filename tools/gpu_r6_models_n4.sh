#!/bin/bash
# Round 6: GPT-2 and ResNet-18 DDP benches at N = 4 with every rank time-sharing the one GPU
# (--shared-gpu: gloo control group, peer route for the gradient buckets) -- a correctness rehearsal of
# the W = 4 model paths (the throughput of time-sliced ranks means nothing).
set -o pipefail
O=gpurun_out/${1:-r6_models_n4}
mkdir -p $O
export TMPDIR=/tmp
for m in gpt2 resnet18; do
  t0=$(date +%s)
  timeout -k 10 500 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 \
    --master-port 2962$([ $m = gpt2 ] && echo 1 || echo 2) bench.py --model $m --gpus 4 --shared-gpu --steps 4 --warmup 2 \
    --bucket-mb 25 > $O/${m}_n4.json 2> $O/${m}_n4.err || { tail -30 $O/${m}_n4.err; exit 1; }
  echo "$m N=4 wall $(( $(date +%s) - t0 )) s" | tee $O/${m}_n4_wall.txt
  head -c 1500 $O/${m}_n4.json; echo
done
