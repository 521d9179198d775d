set -o pipefail
mkdir -p gpurun_out/jit
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_program.py > gpurun_out/jit/pytest.log 2>&1 || { tail -40 gpurun_out/jit/pytest.log; exit 1; }
tail -3 gpurun_out/jit/pytest.log
run() { name=$1; shift; timeout -k 10 180 python bench.py --no-cpu "$@" > gpurun_out/jit/$name.json 2> gpurun_out/jit/$name.err || { echo FAIL $name; tail -5 gpurun_out/jit/$name.err; exit 1; }
  python -c "import json; l=json.loads(open('gpurun_out/jit/$name.json').read().strip().splitlines()[-1]); print('$name', l['value'], l['ms_per_step'], l['roofline']['kernel_ms'])"; }
for w in c2 c4; do
  run ${w}_jit --steps 200 --warmup 20 --workload $w --classify ipclass16
  run ${w}_interp --steps 200 --warmup 20 --workload $w --classify ipclass16 --program-jit 0
done
run drv_jit --gpus 1 --steps 20 --warmup 5 --classify ipclass16
