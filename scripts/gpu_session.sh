#!/bin/bash
# One GPU-box session: parity tests, smoke, short bench. Stops at the first
# step that faults/aborts/times out (exit codes other than 0/1).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name" ; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-all}
[[ $STEPS == *pytest* || $STEPS == all ]] && run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
[[ $STEPS == *smoke* || $STEPS == all ]] && run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $STEPS == *bench* || $STEPS == all ]] && run bench 600 python bench.py ${BENCH_ARGS:---steps 200 --warmup 20}
exit 0
