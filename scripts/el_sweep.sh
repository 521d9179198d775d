#!/bin/bash
# The element over threads x BATCH x SLOTS, interleaved repetitions (one JSON
# line per run): scripts/el_sweep.sh [REPS] [THREADS...] (env BATCHES, SLOTS_LIST)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
reps=${1:-3}; shift
ths=${@:-16 8}
for rep in $(seq 1 $reps); do
  for t in $ths; do
    for b in ${BATCHES:-2048 4096 8192}; do
      for s in ${SLOTS_LIST:-2 3}; do
        timeout -k 5 120 python scripts/element_threads.py $t $b auto $s || exit $?
      done
    done
  done
done
