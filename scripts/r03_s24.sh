#!/bin/bash
# round 3, session 24: the element's default (ZEROCOPY auto, shared queue) at
# 4/8/16 threads with BATCH 4096 / 8192 / 16384, three interleaved rounds.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2 3; do
  for t in 16 8 4; do
    for b in 4096 8192 16384; do
      timeout -k 10 120 python scripts/element_threads.py $t $b > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_batch.log; exit 1; }
      grep threads /tmp/x >> gpurun_out/el_batch.log
    done
  done
done
