#!/bin/bash
# round 3, session 17: the shared zero-copy queue of FCGPU_SPAN_AUTO (several
# contexts' batches in one k_rx launch; RxJob::ctr) -- GPU tests, the element
# at 8/16 threads with ZEROCOPY auto (queue) vs true (a launch per batch),
# interleaved; then the driver command, kernel traces and PMC passes on the
# changed kernel (final script steps bench,kt,pmc).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_c.log 2>&1 || exit $?
for rep in 1 2; do
  for t in 16 8; do
    for b in 4096 16384; do
      for zc in auto true; do
        timeout -k 10 120 python scripts/element_threads.py $t $b $zc > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_agg.log; exit 1; }
        grep threads /tmp/x >> gpurun_out/el_agg.log
      done
    done
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_el16_agg -o run -- python3 scripts/element_threads.py 16 4096 auto > gpurun_out/kt_el16_agg.log 2>&1 || exit $?
STEPS=smoke,bench,kt,pmc bash scripts/r03_final.sh > gpurun_out/final_c.txt 2>&1
