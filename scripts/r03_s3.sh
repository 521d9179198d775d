#!/bin/bash
# round 3, session 3: where the element's host threads spend their time --
# HIP API trace at 1 and 8 threads, and copy-engine / queue variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for t in 1 8; do
  timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -f csv -d gpurun_out/prof_hip$t -o run -- python3 scripts/element_threads.py $t > gpurun_out/hip$t.log 2>&1 || exit $?
done
for t in 1 8 16; do
  HSA_ENABLE_SDMA=0 timeout -k 10 120 python scripts/element_threads.py $t >> gpurun_out/el_nosdma.log 2>&1 || exit $?
done
for q in 1 2 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python scripts/element_threads.py 8 >> gpurun_out/el_q.log 2>&1 || exit $?
done
