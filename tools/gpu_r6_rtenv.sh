#!/bin/bash
# Round 6: HIP runtime settings vs the toy-CNN 20-step window.  Each arm is "name:lead:VAR=VAL,...";
# arms are interleaved, REPS reps each, PDE_BENCH_TRACE=1 (host launch time, event-timed GPU window).
#   bash tools/gpu_r6_rtenv.sh OUTDIR REPS ARM...
set -o pipefail
O=gpurun_out/${1:-r6_rtenv}; REPS=${2:-4}; shift 2
mkdir -p $O
export TMPDIR=/tmp PDE_BENCH_TRACE=1
for r in $(seq 1 $REPS); do
  for arm in "$@"; do
    IFS=: read -r name lead envs <<< "$arm"
    E=(); [ -n "$envs" ] && IFS=, read -r -a E <<< "$envs"
    env "${E[@]}" PDE_BENCH_LEAD=$lead timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure off \
      > $O/w20_${name}_$r.json 2> $O/w20_${name}_$r.err || { tail -20 $O/w20_${name}_$r.err; exit 1; }
  done
done
python3 - $O "$@" <<'PY'
import json, sys, glob, statistics
o = sys.argv[1]
for arm in sys.argv[2:]:
    name = arm.split(":")[0]
    us, gpu, launch = [], [], []
    for f in sorted(glob.glob(f"{o}/w20_{name}_*.json")):
        us.append(json.load(open(f))["ms_per_step"] * 1000)
        for line in open(f[:-5] + ".err"):
            if line.startswith('{"trace_host_us"'):
                t = json.loads(line)
        gpu.append(t["trace_gpu_us"] / 20)
        launch.append(t["trace_launch_us"])
    print(f"{arm:50s} us/step", [round(x, 2) for x in us], "median", round(statistics.median(us), 2),
          "| gpu", round(statistics.median(gpu), 2), "| launch", round(statistics.median(launch), 1))
PY
