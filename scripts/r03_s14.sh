#!/bin/bash
# round 3, session 14: the element's host-side ceiling on the box's CPUs --
# the element harness linked against scripts/mock_fcgpu.cc (results appear at
# once, no GPU work) at 1-16 threads, beside the real element's rates.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for b in 16384 4096; do
  for t in 1 2 4 8 12 16; do
    timeout -k 10 120 ./scripts/mock/element_bench $t $b >> gpurun_out/mock_el.log 2>&1 || exit $?
  done
done
nproc >> gpurun_out/mock_el.log; python3 -c "import os; print('affinity', len(os.sched_getaffinity(0)))" >> gpurun_out/mock_el.log
