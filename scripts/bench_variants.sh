#!/bin/bash
# Bench variants on one GPU box: headline + workload/classifier/flow-table variants.
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
V=${VARIANTS:-c2_lb,c3_lb,c4_lb,c5_lb,c2_ipc16,c4_ipc16,c2_flow,c3_flow,c4_flow,c2_global,c2_noperm,c2_s2,c2_s3}
has() { [[ ",$V," == *",$1,"* ]]; }
has c2_lb && run c2_lb --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
has c3_lb && run c3_lb --workload c3 --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
has c4_lb && run c4_lb --workload c4 --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
has c5_lb && run c5_lb --workload c5 --steps 200 --warmup 20 --no-cpu
has c2_ipc16 && run c2_ipc16 --classify ipclass16 --steps 200 --warmup 20 --no-cpu
has c4_ipc16 && run c4_ipc16 --workload c4 --classify ipclass16 --steps 200 --warmup 20 ${CPU_ARGS:---cpu-seconds 10}
has c2_flow && run c2_flow --flow-capacity 1048576 --steps 200 --warmup 20 --no-cpu
has c3_flow && run c3_flow --workload c3 --flow-capacity 1048576 --steps 200 --warmup 20 --no-cpu
has c4_flow && run c4_flow --workload c4 --flow-capacity 2097152 --steps 200 --warmup 20 --no-cpu
has c2_global && run c2_global --partition global --steps 200 --warmup 20 --no-cpu
has c2_noperm && run c2_noperm --no-perm --steps 200 --warmup 20 --no-cpu
has c2_s2 && run c2_s2 --streams 2 --steps 200 --warmup 20 --no-cpu
has c2_s3 && run c2_s3 --streams 3 --steps 200 --warmup 20 --no-cpu
exit 0
