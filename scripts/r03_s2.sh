#!/bin/bash
# round 3, session 2: GPU tests (RCCL fix), element thread scaling with 16 HW
# queues, a copy/kernel trace of 8 element threads, EA request sizes per config.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_rccl.py tests/test_flow_imp.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || exit $?
for q in 4 16; do
  for t in 1 4 8 16; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python scripts/element_threads.py $t >> gpurun_out/el_q$q.log 2>&1 || exit $?
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -f csv -d gpurun_out/prof_el8 -o run -- python3 scripts/element_threads.py 8 > gpurun_out/el8_trace.log 2>&1 || exit $?
P="--steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1"
for w in c2 c3 c5; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_ea_$w -o run -- python3 bench.py $P --workload $w > gpurun_out/pmc_ea_$w.log 2>&1 || exit $?
done
timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_ea_c4flow -o run -- python3 bench.py --steps 40 --warmup 4 --no-cpu --no-timing --workload c4 --flow-capacity 2000000 > gpurun_out/pmc_ea_c4flow.log 2>&1 || exit $?
