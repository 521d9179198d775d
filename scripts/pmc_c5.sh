#!/bin/bash
# PMC read traffic and L2 requests of k_rx for C5 (VLAN/IPv6 mix) and C2, one batch per launch.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1"
for w in c2 c5 c3; do
  timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_${w}_fetch -o run -- python3 bench.py $B --workload $w > gpurun_out/pmc_${w}_fetch.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_HIT_sum TCC_MISS_sum --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_${w}_ea -o run -- python3 bench.py $B --workload $w > gpurun_out/pmc_${w}_ea.log 2>&1 || exit $?
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_${w}_sq -o run -- python3 bench.py $B --workload $w > gpurun_out/pmc_${w}_sq.log 2>&1 || exit $?
  echo "$w ok"
done
