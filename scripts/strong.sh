# per-GPU shard sizes of the strong (C4, configs[3]) and weak curves on one GPU
set -o pipefail
mkdir -p gpurun_out/strong
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/strong/$name.json 2>/dev/null || { echo FAIL $name; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/strong/$name.json').read().strip().splitlines()[-1]); print('$name', l['value'], l['ms_per_step'], (l['roofline'] or {}).get('kernel_ms'))"; }
for p in 1048576 524288 262144 131072; do
  run drv_c4_$p --gpus 1 --steps 20 --warmup 5 --workload c4 --packets $p
  run long_c4_$p --steps 200 --warmup 20 --workload c4 --packets $p
done
