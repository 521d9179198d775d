#!/bin/bash
# round 3, session 18: the element at 16 threads through the shared zero-copy
# queue (ZEROCOPY auto) with 2 vs 3 slots per thread and 4096 / 8192 packets
# per batch, against ZEROCOPY true; twice, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "16 4096 auto 2" "16 4096 auto 3" "16 8192 auto 3" "16 4096 true 3" "12 4096 auto 3" "4 4096 auto 3"; do
    timeout -k 10 120 python scripts/element_threads.py $cfg > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_q3.log; exit 1; }
    grep threads /tmp/x >> gpurun_out/el_q3.log
  done
done
