#!/bin/bash
# Bench variants on one GPU box: headline + workload/classifier variants.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
set -o pipefail
run() {  # name args...
  local name=$1; shift
  timeout -k 10 300 python bench.py "$@" > "gpurun_out/bv_$name.json" 2> "gpurun_out/bv_$name.err"
  local rc=$?
  echo "== $name rc=$rc"; tail -n 1 "gpurun_out/bv_$name.json"
  if [ $rc -ne 0 ]; then tail -n 5 "gpurun_out/bv_$name.err"; exit $rc; fi
}
run c2_lb --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
run c4_lb --workload c4 --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
run c2_ipc16 --classify ipclass16 --steps 200 --warmup 20 --no-cpu
run c4_ipc16 --workload c4 --classify ipclass16 --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
