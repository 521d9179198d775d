#!/bin/bash
# round 3, session 25: the final tree with BATCH auto -- every GPU test, smoke,
# the driver command, and the element's defaults at 1/2/4/8/12/16 threads twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_e.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_e.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_e.log 2>&1 || exit $?
for rep in 1 2; do
  for t in 1 2 4 8 12 16; do
    timeout -k 10 120 python scripts/element_threads.py $t 0 > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_default.log; exit 1; }
    grep threads /tmp/x >> gpurun_out/el_default.log
  done
done
