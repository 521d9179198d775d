#!/bin/bash
# round 3, session 8: GPU tests on the zero-copy element mode; the element's
# host rate with ZEROCOPY false/true at 1-16 threads; PCIe microbenchmarks
# (H2D copy rate by size x streams; zero-copy reads of packed 64-B records vs
# scattered pieces); the driver command once.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
for b in 16384 4096; do
  for t in 1 4 8 16; do
    for zc in 0 1; do
      timeout -k 10 120 python scripts/element_threads.py $t $b $zc > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_zc.log; exit 1; }
      grep threads /tmp/x >> gpurun_out/el_zc.log
    done
  done
done
timeout -k 10 120 ./scripts/kcopy > gpurun_out/kcopy.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/khostgather 262144 2304 1 > gpurun_out/khg_scattered.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/khostgather 262144 64 0 > gpurun_out/khg_packed.log 2>&1 || exit $?
timeout -k 10 120 python bench.py > gpurun_out/bench.log 2>&1 || exit $?
