#!/bin/bash
# A/B of two builds of the element harness on the GPU box: the in-tree
# libfcclick.so against $ALT (FCCLICK_LIB), interleaved repetitions:
#   ALT=scripts/mock/nt_real/libfcclick.so scripts/el_ab_lib.sh [REPS]
# (ALT_FCGPU: also another libfcgpu.so -- the alternate harness must be linked
# against that same file)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq 1 ${1:-3}); do
  for t in 16 8; do
    for b in 0 8192; do
      for v in base alt; do
        echo -n "{\"lib\": \"$v\", \"r\": "
        if [ $v = alt ]; then FCGPU_LIB=$ALT_FCGPU FCCLICK_LIB=$ALT timeout -k 5 120 python scripts/element_threads.py $t $b auto 2 || exit $?
        else timeout -k 5 120 python scripts/element_threads.py $t $b auto 2 || exit $?; fi
        echo "}"
      done
    done
  done
done
