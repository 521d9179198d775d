# A/B on one box: the driver's 20-step line with input-only prefault (1) vs
# inputs + output sets (2), alternated
set -o pipefail
mkdir -p gpurun_out/pfab
for i in 1 2 3 4 5; do
  for pf in 1 2; do
    timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --prefault $pf \
      > gpurun_out/pfab/pf${pf}_$i.json 2>/dev/null || exit 1
    python -c "import json; l=json.loads(open('gpurun_out/pfab/pf${pf}_$i.json').read().strip().splitlines()[-1]); print('pf$pf', l['value'], l['ms_per_step'], l['roofline']['kernel_ms'])"
  done
done
