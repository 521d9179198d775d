set -o pipefail
mkdir -p gpurun_out/drv
for i in 1 2 3 4 5 6; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv/b$i.json 2> gpurun_out/drv/b$i.err || exit 1
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --timing-every 10 --no-cpu > gpurun_out/drv/old$i.json 2> gpurun_out/drv/old$i.err || exit 1
done
for f in gpurun_out/drv/*.json; do python -c "import json; l=json.loads(open('$f').read().strip().splitlines()[-1]); r=l['roofline']; print('$f', l['value'], l['ms_per_step'], r['frac'], r.get('kernel_ms'), r.get('sampled_launches'))"; done
