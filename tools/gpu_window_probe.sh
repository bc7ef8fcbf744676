set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 120 python tools/window_probe.py > gpurun_out/wp$i.json 2>/dev/null || exit 1
cat gpurun_out/wp$i.json
PDE_BENCH_TRACE=1 timeout -k 10 120 python bench.py --steps 20 --warmup 5 --comm-figure off > gpurun_out/wpb$i.json 2> gpurun_out/wpb$i.err || exit 1
python -c "import json;print(json.load(open('gpurun_out/wpb$i.json'))['ms_per_step'])"; grep trace gpurun_out/wpb$i.err
done
