set -o pipefail
mkdir -p gpurun_out/nb
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/nb/$name.json 2>/dev/null || { echo FAIL $name; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/nb/$name.json').read().strip().splitlines()[-1]); print('$name', l['value'], l['ms_per_step'], l['config']['hbm_batches'])"; }
for v in "--workload c3" "--frame-bytes 512" "--frame-bytes 128" "--frame-bytes 1500" "--workload c5" ""; do
  n=$(echo "x$v" | tr -d ' -' | cut -c1-30)
  run f_$n --steps 200 --warmup 20 $v
  run u_$n --steps 200 --warmup 20 --streams 2 --fuse 1 $v
done
