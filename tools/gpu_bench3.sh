#!/bin/bash
# Driver-config bench three times (+ the W=1 comm figure once): step time spread on one box.
set -o pipefail
O=gpurun_out/${1:-bench3}
mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off > $O/bw$i.json 2> $O/bw$i.err || exit 1
  python -c "import json;d=json.load(open('$O/bw$i.json'));print(d['ms_per_step'])"
done
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bw_fc.json 2> $O/bw_fc.err || exit 1
python -c "import json;d=json.load(open('$O/bw_fc.json'));print(d['ms_per_step'], d['w1_rccl_comm'].get('ms_per_step'), d['w1_rccl_comm'].get('schedule'))"
