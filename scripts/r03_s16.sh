#!/bin/bash
# round 3, session 16: the speculative strided window gather of zero-copy
# submissions (RxArgs::stride64) -- GPU tests (hit and miss paths), then A/B
# against the previous build (lib/ab/: no speculation), interleaved: the
# driver command (device-resident: the flag is off, the kernel gains one
# uniform branch), the host-resident ring and the element at 16 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
AB="FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu.so FCCLICK_LIB=fastclick_amd/lib/ab/libfcclick.so"
timeout -k 10 300 python -u -m pytest tests/test_span_modes.py tests/test_element.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_spec.log 2>&1 || exit $?
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/drv_spec$rep.log 2>&1 || exit $?
  env $AB timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/drv_nospec$rep.log 2>&1 || exit $?
done
for rep in 1 2; do
  timeout -k 10 300 python scripts/host_rate.py span > gpurun_out/span_spec$rep.log 2>&1 || exit $?
  env $AB timeout -k 10 300 python scripts/host_rate.py span > gpurun_out/span_nospec$rep.log 2>&1 || exit $?
  for b in 4096 16384; do
    timeout -k 10 120 python scripts/element_threads.py 16 $b true > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_spec.log; exit 1; }
    echo "spec $(grep threads /tmp/x)" >> gpurun_out/el_spec.log
    env $AB timeout -k 10 120 python scripts/element_threads.py 16 $b true > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_spec.log; exit 1; }
    echo "nospec $(grep threads /tmp/x)" >> gpurun_out/el_spec.log
  done
done
for zc in 1; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_el1_spec -o run -- python3 scripts/element_threads.py 1 4096 $zc > gpurun_out/kt_el1_spec.log 2>&1 || exit $?
done
