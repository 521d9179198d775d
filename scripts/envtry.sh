set -o pipefail
mkdir -p gpurun_out/env
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu --gpus 1 --steps 20 --warmup 5 > gpurun_out/env/$name.json 2>/dev/null || { echo FAIL $name; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/env/$name.json').read().strip().splitlines()[-1]); print('$name', l['value'], l['ms_per_step'], l['roofline']['kernel_ms'])"; }
for i in 1 2 3; do
  run base_$i
  HIP_FORCE_DEV_KERNARG=1 run devka_$i
done
