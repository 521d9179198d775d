#!/bin/bash
# round 3, session 10 (= session 9 + element slots): line-request sizes -- klines (64-B pieces packed vs
# alone in their 128-B line, five cache policies) timed and under a PMC pass
# (EA read requests by size); C2/C3/C5 k_rx request sizes; the 1/8 strong
# shard (131,072 packets, 122 rotating copies) with FETCH_SIZE.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 ./scripts/klines > gpurun_out/klines.log 2>&1 || exit $?
timeout -s KILL 60 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum -f csv -d gpurun_out/pmc_klines -o run -- ./scripts/klines 262144 > gpurun_out/pmc_klines.log 2>&1 || exit $?
P="--steps 20 --warmup 2 --no-cpu --no-timing --streams 1 --fuse 1"
for w in c2 c3 c5; do
  timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_sum --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_rq_$w -o run -- python3 bench.py $P --workload $w > gpurun_out/pmc_rq_$w.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --workload c4 --shard strong --packets 131072 > gpurun_out/strong131k.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --workload c4 --shard strong --packets 131072 > gpurun_out/strong131k_200.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_strong131k -o run -- python3 bench.py --steps 40 --warmup 2 --no-cpu --no-timing --workload c4 --shard strong --packets 131072 > gpurun_out/pmc_strong131k.log 2>&1 || exit $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_rx -f csv -d gpurun_out/pmc_strong131k_w -o run -- python3 bench.py --steps 40 --warmup 2 --no-cpu --no-timing --workload c4 --shard strong --packets 131072 > gpurun_out/pmc_strong131k_w.log 2>&1 || exit $?
# the element: ZEROCOPY with 2 or 3 slots, 16 threads, batch sizes; a kernel trace
timeout -k 10 300 python -u -m pytest tests/test_element.py -m gpu -x -q --timeout 120 --timeout-method thread -k zerocopy > gpurun_out/pytest_zc.log 2>&1 || exit $?
for rep in 1 2; do
  for cfg in "16 2048 1 2" "16 2048 1 3" "16 4096 1 2" "16 4096 1 3" "16 8192 1 3" "8 4096 1 3" "1 16384 1 3" "1 16384 0 3" "1 16384 0 2"; do
    timeout -k 10 120 python scripts/element_threads.py $cfg > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_slots.log; exit 1; }
    grep threads /tmp/x >> gpurun_out/el_slots.log
  done
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_el16 -o run -- python3 scripts/element_threads.py 16 4096 1 3 > gpurun_out/kt_el16.log 2>&1 || exit $?
