#!/bin/bash
# round 3, session 15 (final part B): GPU tests on the final library; the
# element at 16 threads, zero-copy, with 4 / 8 / 16 HW queues
# (GPU_MAX_HW_QUEUES, 4 = HIP's default on the box); then the final
# script's variants, frame-size sweep and host-resident steps.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_b.log 2>&1 || exit $?
for rep in 1 2; do
  for q in 4 8 16; do
    for b in 4096 16384; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python scripts/element_threads.py 16 $b true > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_hwq.log; exit 1; }
      grep threads /tmp/x >> gpurun_out/el_hwq.log
    done
  done
done
STEPS=variants,sweep,host bash scripts/r03_final.sh > gpurun_out/final_b.txt 2>&1
