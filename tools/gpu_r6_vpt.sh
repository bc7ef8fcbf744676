#!/bin/bash
# Round 6: in-place one-shot vectors per thread (PDE_PEER_IP_VPT = 1 / 2 / 4) after the barrier B / C
# change, read from the W = 1 comm figure's route and schedule tables; interleaved, one box.
set -o pipefail
O=gpurun_out/${1:-r6_vpt}
mkdir -p $O
export TMPDIR=/tmp
for r in 1 2 3; do
  for v in 1 2 4; do
    PDE_PEER_IP_VPT=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --comm-figure on \
      > $O/vpt${v}_$r.json 2>> $O/err.txt || { tail -20 $O/err.txt; exit 1; }
  done
done
python3 - $O <<'PY'
import json, sys, glob, statistics
o = sys.argv[1]
for v in (1, 2, 4):
    call, serial = [], []
    for f in sorted(glob.glob(f"{o}/vpt{v}_*.json")):
        c = json.load(open(f))["w1_rccl_comm"]
        call.append(c["route_us_per_call"]["431296"]["peer1"])
        serial.append(c["schedule_us_per_step"]["serial 431296:peer1"] - c["compute_only_us_per_step"])
    print("vpt", v, "peer1 call", call, "median", statistics.median(call), "| serial peer1 - co",
          [round(x, 2) for x in serial], "median", round(statistics.median(serial), 2))
PY
