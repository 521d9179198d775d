#!/bin/bash
# round 3, session 5: element tests after the per-tile annotate+emit change,
# then the element thread sweep.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_element.py tests/test_rewrite.py tests/test_flow.py tests/test_flow_imp.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_el.log 2>&1 || exit $?
for t in 1 2 4 8 16; do
  timeout -k 10 120 python scripts/element_threads.py $t >> gpurun_out/el_tile.log 2>&1 || exit $?
done
for t in 1 4 8 16; do
  timeout -k 10 120 python scripts/element_threads.py $t 8192 >> gpurun_out/el_tile.log 2>&1 || exit $?
done
