#!/bin/bash
# Round 6: the toy-CNN headline's 20-step window with one lead step (a 1-step hipGraph replayed ahead of
# the 19-step graph; bench.py default) against one 20-step graph (PDE_BENCH_LEAD=0): interleaved reps
# with PDE_BENCH_TRACE=1 (host window, host launch time, event-timed GPU window on stderr), two 2000-step
# pairs, and an N = 2 shared-GPU rehearsal of the default.
set -o pipefail
O=gpurun_out/${1:-r6_lead}
mkdir -p $O
export TMPDIR=/tmp PDE_BENCH_TRACE=1
for r in 1 2 3 4 5 6 7 8; do
  for v in base lead; do
    L=1; [ $v = base ] && L=0
    PDE_BENCH_LEAD=$L timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/w20_${v}_$r.json 2> $O/w20_${v}_$r.err || exit 1
  done
done
for r in 1 2; do
  for v in base lead; do
    L=1; [ $v = base ] && L=0
    PDE_BENCH_LEAD=$L timeout -k 10 200 python bench.py --steps 2000 --warmup 200 --comm-figure off > $O/w2000_${v}_$r.json 2> $O/w2000_${v}_$r.err || exit 1
  done
done
unset PDE_BENCH_TRACE
timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29617 bench.py --gpus 2 --shared-gpu --steps 20 --warmup 5 > $O/n2_shared.json 2> $O/n2_shared.err || exit 1
python3 - $O <<'PY'
import json, sys, glob, statistics
o = sys.argv[1]
for w, n in (("w20", 20), ("w2000", 2000)):
    for v in ("base", "lead"):
        us, gpu, launch = [], [], []
        for f in sorted(glob.glob(f"{o}/{w}_{v}_*.json")):
            us.append(json.load(open(f))["ms_per_step"] * 1000)
            for line in open(f[:-5] + ".err"):
                if line.startswith('{"trace_host_us"'):
                    t = json.loads(line)
            gpu.append(t["trace_gpu_us"] / n)
            launch.append(t["trace_launch_us"])
        print(w, v, "us/step", [round(x, 2) for x in us], "median", round(statistics.median(us), 2),
              "| gpu us/step median", round(statistics.median(gpu), 2), "| host launch us median", round(statistics.median(launch), 1))
d = json.load(open(f"{o}/n2_shared.json"))
print("n2_shared", d["value"], d["n_gpus"], d["config"]["mode"], d["config"].get("schedule", d["config"].get("grad_allreduce")))
PY
