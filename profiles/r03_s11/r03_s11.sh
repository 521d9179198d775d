#!/bin/bash
# round 3, session 11: GPU tests + smoke on the element's SLOTS / ZEROCOPY auto
# code; the driver command and 200 steps, A/B against a build whose k_rx reads
# the descriptors non-temporally (lib/ab/libfcgpu_descnt.so), interleaved;
# the element's default (ZEROCOPY auto) at 1-16 threads.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || exit $?
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/drv_base$rep.log 2>&1 || exit $?
  FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu_descnt.so timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu > gpurun_out/drv_descnt$rep.log 2>&1 || exit $?
done
for rep in 1 2; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/long_base$rep.log 2>&1 || exit $?
  FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu_descnt.so timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu > gpurun_out/long_descnt$rep.log 2>&1 || exit $?
done
for b in 16384 4096; do
  for t in 1 2 4 8 12 16; do
    timeout -k 10 120 python scripts/element_threads.py $t $b auto > /tmp/x 2>&1 || { cat /tmp/x >> gpurun_out/el_auto.log; exit 1; }
    grep threads /tmp/x >> gpurun_out/el_auto.log
  done
done
