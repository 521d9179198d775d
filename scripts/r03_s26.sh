#!/bin/bash
# round 3, session 26: span-mode / shared-queue GPU tests (programs and a flow
# table among the queue's contexts).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_span_modes.py tests/test_element.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_span2.log 2>&1 || exit $?
