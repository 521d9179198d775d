# with-errors mixes and the cache-resident line, 200 steps each
set -o pipefail
mkdir -p gpurun_out/errvar
B="python bench.py --steps 200 --warmup 20 --no-cpu"
run() { name=$1; shift; timeout -k 10 180 $B "$@" > gpurun_out/errvar/$name.json 2> gpurun_out/errvar/$name.err || { echo "FAIL $name"; exit 1; }; }
run c2_err1 --errors 0.01
run c4_err1 --workload c4 --errors 0.01
run c2_err1_s1 --errors 0.01 --streams 1
run c2_allvalid
run c2_mall --nbuf 1
run c2_mall_s1 --nbuf 1 --streams 1
for f in gpurun_out/errvar/*.json; do python -c "import json,sys; l=json.loads(open('$f').read().strip().splitlines()[-1]); print('$f', l['value'], l['ms_per_step'], l['roofline']['frac'], l['roofline'].get('kernel_ms'), l['config'].get('valid_fraction'))"; done
