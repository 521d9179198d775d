#!/bin/bash
# Timed-region A/B of the driver command (FCGPU_BENCH_DIAG=1: the region
# repeated in-process, enqueue time). Each run under its own time limit; stops
# at the first run that faults or times out.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
DRV="--gpus 1 --steps 20 --warmup 5 --no-cpu"
run() {  # name env... -- args...
  local name=$1; shift
  local envs=()
  while [ "$1" != "--" ]; do envs+=("$1"); shift; done; shift
  env FCGPU_BENCH_DIAG=1 "${envs[@]}" timeout -k 10 300 python bench.py $DRV "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep -h '"diag"' gpurun_out/$name.log)"
  grep -h '"metric"' "gpurun_out/$name.log" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("   value", d["value"], "ms_per_step", d["ms_per_step"], "kernel_ms", (d["roofline"] or {}).get("kernel_ms"))' || true
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
for k in ${AB_RUNS:-1 2 3}; do
  run base$k --
  run kdev0_$k HIP_FORCE_DEV_KERNARG=0 --
  run notime$k -- --no-timing
done
exit 0
