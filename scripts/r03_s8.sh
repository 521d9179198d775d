#!/bin/bash
# round 3, session 8: PCIe microbenchmarks for the element's host path --
# H2D copy rate by size and stream count; zero-copy reads of packed 64-B
# records vs scattered pieces.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 120 ./scripts/kcopy > gpurun_out/kcopy.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/khostgather 262144 2304 1 > gpurun_out/khg_scattered.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/khostgather 262144 64 0 > gpurun_out/khg_packed.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/khostgather 1048576 64 0 > gpurun_out/khg_packed1m.log 2>&1 || exit $?
timeout -k 10 60 ./scripts/khostgather 262144 128 0 > gpurun_out/khg_128.log 2>&1 || exit $?
