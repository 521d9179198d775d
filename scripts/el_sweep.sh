#!/bin/bash
# The element at 8/16 threads over BATCH x SLOTS, interleaved repetitions
# (one JSON line per run): scripts/el_sweep.sh [REPS]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq 1 ${1:-3}); do
  for t in 16 8; do
    for b in 2048 4096 8192; do
      for s in 2 3; do
        timeout -k 5 120 python scripts/element_threads.py $t $b auto $s || exit $?
      done
    done
  done
done
