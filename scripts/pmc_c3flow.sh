#!/bin/bash
# PMC read/write requests of k_rx for C3 with and without the 20k-capacity
# flow table (one batch per launch), each pass its own rocprofv3 run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1 --workload c3"
for v in base flow; do
  X=""; [ $v = flow ] && X="--flow-capacity 20000"
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_c3_$v -o run -- python3 bench.py $B $X > gpurun_out/pmc_c3_$v.log 2>&1 || exit $?
  echo "pmc_c3_$v ok"
done
