#!/bin/bash
# round 3, session 7: the element's span streams -- a stream per slot (default),
# per context, or a few shared by the process (FCGPU_SPAN_STREAMS), 8 and 16 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_element.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_el.log 2>&1 || exit $?
FCGPU_SPAN_STREAMS=shared:2 timeout -k 10 300 python -u -m pytest tests/test_element.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_el_shared.log 2>&1 || exit $?
for rep in 1 2; do
  for mode in slot ctx shared:1 shared:2 shared:4; do
    for t in 8 16; do
      FCGPU_SPAN_STREAMS=$mode timeout -k 10 120 python scripts/element_threads.py $t > /tmp/x 2>&1 || exit $?
      echo "$mode $(grep threads /tmp/x)" >> gpurun_out/streams.log
    done
  done
done
FCGPU_SPAN_STREAMS=shared:2 timeout -k 10 180 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace -f csv -d gpurun_out/tr8s2 -o run -- python3 scripts/element_threads.py 8 > gpurun_out/tr8s2.log 2>&1
