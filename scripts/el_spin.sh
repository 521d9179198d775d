#!/bin/bash
# The element at 16 / 8 threads: runtime waits vs spinning waits
# (FCGPU_SPAN_WAIT=spin), SLOTS 2 and 3, interleaved repetitions.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq 1 ${1:-3}); do
  for t in 16 8; do
    for s in 2 3; do
      for w in block spin; do
        echo -n "{\"wait\": \"$w\", \"r\": "
        FCGPU_SPAN_WAIT=$w timeout -k 5 120 python scripts/element_threads.py $t 0 auto $s || exit $?
        echo "}"
      done
    done
  done
done
