# fused k_rx launches: GPU tests, then the driver command and long runs with/without fusion
set -o pipefail
mkdir -p gpurun_out/fuse
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests > gpurun_out/fuse/pytest.log 2>&1 || { tail -30 gpurun_out/fuse/pytest.log; exit 1; }
tail -2 gpurun_out/fuse/pytest.log
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/fuse/$name.json 2> gpurun_out/fuse/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/fuse/$name.err; exit 1; }; }
for i in 1 2 3 4; do run drv_f24_s2_$i --gpus 1 --steps 20 --warmup 5; done
for i in 1 2 3 4; do run drv_f24_s1_$i --gpus 1 --steps 20 --warmup 5 --streams 1; done
for i in 1 2; do run drv_f1_s2_$i --gpus 1 --steps 20 --warmup 5 --fuse 1; done
run long_f24_s2 --steps 200 --warmup 20
run long_f24_s1 --steps 200 --warmup 20 --streams 1
run long_f1_s2 --steps 200 --warmup 20 --fuse 1
for f in gpurun_out/fuse/*.json; do python -c "import json; l=json.loads(open('$f').read().strip().splitlines()[-1]); r=l['roofline']; print('$f', l['value'], l['ms_per_step'], r['frac'], r.get('kernel_ms'), r.get('sampled_launches'), l['config'].get('batches_per_launch'))"; done
