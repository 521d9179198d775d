#!/bin/bash
# round 3, session 6: A/B of the element's completion (whole-batch annotate,
# then link: lib/ab/libfcclick_old.so; per-tile annotate + link: the current
# build), interleaved, and one full trace at 8 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for t in 1 4 8 16; do
    FCCLICK_LIB=fastclick_amd/lib/ab/libfcclick_old.so timeout -k 10 120 python scripts/element_threads.py $t > /tmp/x 2>&1 || exit $?
    echo "old $(grep threads /tmp/x)" >> gpurun_out/ab.log
    timeout -k 10 120 python scripts/element_threads.py $t > /tmp/x 2>&1 || exit $?
    echo "new $(grep threads /tmp/x)" >> gpurun_out/ab.log
  done
done
timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -f csv -d gpurun_out/tr8 -o run -- python3 scripts/element_threads.py 8 > gpurun_out/tr8.log 2>&1
