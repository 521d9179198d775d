#!/bin/bash
# Element host-side ceiling A/B on the GPU box's CPUs (no GPU used): the
# harness element linked against scripts/mock_fcgpu.cc, variants prebuilt under
# scripts/mock/<variant>/ (element_bench THREADS BATCH REPS -> JSON line).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for t in 1 8 16; do
    b=4096; [ $t = 1 ] && b=16384
    for v in ${VARIANTS:-base}; do
      echo "{\"variant\": \"$v\", \"rep\": $rep, \"r\": $(timeout -k 5 120 scripts/mock/$v/element_bench $t $b 40)}"
    done
  done
done
