#!/bin/bash
# round 3, session 21: the final tree -- every GPU test, smoke, the driver
# command twice (the first with the CPU baseline), the element's default at
# 16 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_final.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_final1.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_final2.log 2>&1 || exit $?
for b in 4096 16384; do
  timeout -k 10 120 python scripts/element_threads.py 16 $b > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_final.log; exit 1; }
  grep threads /tmp/x >> gpurun_out/el_final.log
done
