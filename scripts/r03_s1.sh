#!/bin/bash
# round 3, session 1: kernarg probe, counter list, GPU tests, smoke, driver
# command with and without the plan path (A/B, twice), element thread sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 60 ./scripts/kargs > gpurun_out/kargs.log 2>&1
timeout -k 10 60 rocprofv3 --list-avail > gpurun_out/avail.txt 2>&1
STEPS=tests,smoke bash scripts/session.sh || exit $?
for k in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_plan$k.log 2>&1 || exit $?
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --no-plan > gpurun_out/bench_noplan$k.log 2>&1 || exit $?
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --shard strong --packets 131072 > gpurun_out/bench_strong131k.log 2>&1 || exit $?
timeout -k 10 600 python scripts/host_rate.py threads > gpurun_out/threads.log 2>&1
