#!/bin/bash
# round 3, session 19: pcap ingress GPU tests; the host-resident rates with
# the parallel mapped pcap index (host_rate.py main: pcap 1/4 reader threads,
# mapped 1/4/8 index threads, mbuf, process_host, element).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_pcap.py tests/test_span_modes.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_pcap.log 2>&1 || exit $?
timeout -k 10 600 python scripts/host_rate.py > gpurun_out/host_rate.log 2>&1 || exit $?
