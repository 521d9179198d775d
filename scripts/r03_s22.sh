#!/bin/bash
# round 3, session 22: the whole-batch partition's scatter pass with every
# tile's inputs loaded up front -- partition GPU tests, then A/B against the
# previous build (lib/ab/libfcgpu.so), interleaved: --partition global at 200
# steps and the driver command, and the default driver command (k_rx alone).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_parity_gpu.py tests/test_golden.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_part.log 2>&1 || exit $?
AB="FCGPU_LIB=fastclick_amd/lib/ab/libfcgpu.so"
for rep in 1 2 3; do
  timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu --partition global > gpurun_out/glob_new$rep.log 2>&1 || exit $?
  env $AB timeout -k 10 120 python bench.py --steps 200 --warmup 20 --no-cpu --partition global > gpurun_out/glob_old$rep.log 2>&1 || exit $?
  timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --partition global > gpurun_out/glob20_new$rep.log 2>&1 || exit $?
  env $AB timeout -k 10 120 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu --partition global > gpurun_out/glob20_old$rep.log 2>&1 || exit $?
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/kt_glob -o run -- python3 bench.py --steps 40 --warmup 4 --no-cpu --no-timing --partition global > gpurun_out/kt_glob.log 2>&1 || exit $?
