#!/bin/bash
# Host-resident pipeline sweep over chunk sizes (PCIe-inclusive rates).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for ch in 32768 65536 131072 262144; do
  FCGPU_HOST_CHUNK=$ch timeout -k 10 240 python scripts/host_rate.py > gpurun_out/host_rate_$ch.json 2> gpurun_out/host_rate_$ch.err || exit $?
  cat gpurun_out/host_rate_$ch.json
done
