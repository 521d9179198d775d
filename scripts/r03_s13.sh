#!/bin/bash
# round 3, session 13: span-mode GPU tests (block and span submissions, copy /
# zero-copy / auto); the host-resident ring rate (fcgpu_span_submit, no
# per-packet host work) with copies vs zero-copy at 1M/256K/64K packets per
# submission; a kernel trace of the 1M zero-copy case.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_span_modes.py tests/test_element.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_span.log 2>&1 || exit $?
timeout -k 10 300 python scripts/host_rate.py span > gpurun_out/span.log 2>&1 || exit $?
timeout -k 10 300 python scripts/host_rate.py span > gpurun_out/span2.log 2>&1 || exit $?
