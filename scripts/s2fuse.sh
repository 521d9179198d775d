# fused launches on one vs two streams
set -o pipefail
mkdir -p gpurun_out/s2f
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/s2f/$name.json 2>/dev/null || { echo FAIL $name; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/s2f/$name.json').read().strip().splitlines()[-1]); print('$name', l['value'], l['ms_per_step'])"; }
for i in 1 2 3; do run drv_s1_$i --gpus 1 --steps 20 --warmup 5; run drv_s2f_$i --gpus 1 --steps 20 --warmup 5 --streams 2; done
for v in "--frame-bytes 512" "--workload c3" "--classify ipclass16" ""; do
  n=$(echo "x$v" | tr -d ' -' | cut -c1-30)
  run l_s1_$n --steps 200 --warmup 20 $v
  run l_s2f_$n --steps 200 --warmup 20 --streams 2 $v
  run l_s2u_$n --steps 200 --warmup 20 --streams 2 --fuse 1 $v
  run l_s3f_$n --steps 200 --warmup 20 --streams 3 $v
done
