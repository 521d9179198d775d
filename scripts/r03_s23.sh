#!/bin/bash
# round 3, session 23: the final tree -- every GPU test, smoke, the driver
# command 3x (the first with the CPU baseline) and 200 steps, kernel traces,
# the PMC passes behind profiles/pmc_traffic.json (final script steps), and
# the element's default at 16 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=tests,smoke,bench,kt,pmc bash scripts/r03_final.sh > gpurun_out/final_d.txt 2>&1 || exit $?
for b in 4096 16384; do
  timeout -k 10 120 python scripts/element_threads.py 16 $b > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_final.log; exit 1; }
  grep threads /tmp/x >> gpurun_out/el_final.log
done
