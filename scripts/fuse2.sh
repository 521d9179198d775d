set -o pipefail
mkdir -p gpurun_out/fuse2
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_parity_gpu.py > gpurun_out/fuse2/pytest.log 2>&1 || { tail -30 gpurun_out/fuse2/pytest.log; exit 1; }
tail -1 gpurun_out/fuse2/pytest.log
run() { name=$1; shift; timeout -k 10 120 python bench.py --no-cpu "$@" > gpurun_out/fuse2/$name.json 2> gpurun_out/fuse2/$name.err || { echo "FAIL $name"; tail -5 gpurun_out/fuse2/$name.err; exit 1; }; }
run long_f24_s1 --steps 200 --warmup 20 --streams 1
run long_f24_s2 --steps 200 --warmup 20
run long_f1_s2 --steps 200 --warmup 20 --fuse 1
run long_f4_s2 --steps 200 --warmup 20 --fuse 4
run long_f2_s2 --steps 200 --warmup 20 --fuse 2
for i in 1 2; do run drv_f24_s1_$i --gpus 1 --steps 20 --warmup 5 --streams 1; done
for f in gpurun_out/fuse2/*.json; do python -c "import json; l=json.loads(open('$f').read().strip().splitlines()[-1]); r=l['roofline']; print('$f', l['value'], l['ms_per_step'], r['frac'], r.get('kernel_ms'), r.get('sampled_launches'), l['config'].get('batches_per_launch'))"; done
