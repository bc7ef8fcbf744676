set -o pipefail
mkdir -p gpurun_out
(rocm-smi --showproductname --showmeminfo vram 2>&1 | head -30) > gpurun_out/probe_smi.txt || true
timeout -k 10 300 python tools/ref_baseline.py --mode faithful --steps 300 --warmup 50 > gpurun_out/base_faithful.json 2>gpurun_out/base_faithful.err &&
timeout -k 10 300 python tools/ref_baseline.py --mode nosync --steps 300 --warmup 50 > gpurun_out/base_nosync.json 2>gpurun_out/base_nosync.err &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29511 tools/ref_baseline.py --dist --mode faithful --steps 300 --warmup 50 > gpurun_out/base_dist1.json 2>gpurun_out/base_dist1.err
echo "baseline done rc=$?"
timeout -k 10 120 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29512 tools/rccl_two_ranks_one_gpu.py > gpurun_out/rccl2.txt 2>&1; echo "rccl2 rc=$?" >> gpurun_out/rccl2.txt
cat gpurun_out/*.json; tail -5 gpurun_out/rccl2.txt
