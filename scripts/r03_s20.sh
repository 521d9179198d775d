#!/bin/bash
# round 3, session 20: pcap ingress with the parallel mapped index (stricter
# speculative starts), 1-8 index threads, twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pcap.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pcap2.log 2>&1 || exit $?
timeout -k 10 600 python scripts/host_rate.py pcap > gpurun_out/pcap_rates.log 2>&1 || exit $?
