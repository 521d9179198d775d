#!/bin/bash
# round 3, session 12: span modes GPU test; strong-shard rows at the N=2 and
# N=4 shard sizes (shard-only arenas, >= 1.15 GB rotation); kernel traces of
# one element thread, copy vs zero-copy (k_rx duration of a 4096-packet batch
# read from device memory vs over PCIe).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_span_modes.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_span.log 2>&1 || exit $?
for p in 524288 262144; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --workload c4 --shard strong --packets $p > gpurun_out/strong${p}.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --gpus 1 --steps 200 --warmup 5 --no-cpu --workload c4 --shard strong --packets $p > gpurun_out/strong${p}_200.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --workload c4 --shard strong > gpurun_out/strong1048576.log 2>&1 || exit $?
for zc in 0 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_el1_zc$zc -o run -- python3 scripts/element_threads.py 1 4096 $zc > gpurun_out/kt_el1_zc$zc.log 2>&1 || exit $?
done
