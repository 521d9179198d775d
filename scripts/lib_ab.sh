#!/bin/bash
# Same-box A/B of two builds of libfcgpu.so (FCGPU_LIB): each bench variant
# alternately on A (fastclick_amd/lib/ab/libfcgpu_a.so) and B (the in-tree
# library), AB_ROUNDS times. Each run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
A=fastclick_amd/lib/ab/libfcgpu_a.so
B=fastclick_amd/lib/libfcgpu.so
IFS=';' read -ra VARS <<< "${AB_VARIANTS:---flow-capacity 1;--workload c3 --flow-capacity 20000;--workload c4 --flow-capacity 2000000;}"
for r in $(seq 1 ${AB_ROUNDS:-2}); do
  for v in "${VARS[@]}"; do
    for lib in A B; do
      L=$A; [ $lib = B ] && L=$B
      n=$(echo "$v" | tr -d ' -' | cut -c1-40)
      FCGPU_LIB=$L timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu $v > gpurun_out/ab_${lib}_${n:-c2}_$r.log 2>&1 || exit $?
      echo "$lib r$r [$v] $(grep -o '"value": [0-9.]*' gpurun_out/ab_${lib}_${n:-c2}_$r.log) $(grep -o '"kernel_ms": [0-9.]*' gpurun_out/ab_${lib}_${n:-c2}_$r.log)"
    done
  done
done
