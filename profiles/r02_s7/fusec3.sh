set -o pipefail
mkdir -p gpurun_out/fc3
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/fc3/$name.json 2>/dev/null || { echo FAIL $name; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/fc3/$name.json').read().strip().splitlines()[-1]); print('$name', l['value'], l['ms_per_step'], (l['roofline'] or {}).get('kernel_ms'))"; }
for f in 1 2 4 24; do run s1_f$f --steps 200 --warmup 20 --workload c3 --fuse $f; run s2_f$f --steps 200 --warmup 20 --workload c3 --fuse $f --streams 2; done
run s1_f24_nt --steps 200 --warmup 20 --workload c3 --no-timing
run s2_f1_nt --steps 200 --warmup 20 --workload c3 --fuse 1 --streams 2 --no-timing
run s1_f24_nb1 --steps 200 --warmup 20 --workload c3 --nbuf 2
run s2_f1_nb1 --steps 200 --warmup 20 --workload c3 --fuse 1 --streams 2 --nbuf 2
