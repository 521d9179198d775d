#!/bin/bash
# GPU-box session: tests, bench, rocprofv3 kernel trace + PMC passes, host-resident
# rate. Each GPU step has its own time limit; stop at the first fault/abort/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc"; tail -n 4 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
S=${STEPS:-tests,bench,ktrace,pmc,host}
B="--steps 200 --warmup 20"
[[ $S == *tests* ]] && step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
[[ $S == *smoke* ]] && step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
[[ $S == *bench* ]] && step bench 600 python bench.py $B
[[ $S == *ktrace* ]] && step ktrace 600 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof_ktrace -o run -- python3 bench.py $B --no-cpu
[[ $S == *pmc* ]] && step pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex k_rx -f csv -d gpurun_out/prof_fetch -o run -- python3 bench.py --steps 40 --warmup 4 --no-cpu --no-timing
[[ $S == *pmc* ]] && step pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex k_rx -f csv -d gpurun_out/prof_write -o run -- python3 bench.py --steps 40 --warmup 4 --no-cpu --no-timing
[[ $S == *pmc* ]] && step pmc_ea 600 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --kernel-include-regex k_rx -f csv -d gpurun_out/prof_ea -o run -- python3 bench.py --steps 40 --warmup 4 --no-cpu --no-timing
[[ $S == *host* ]] && step host_rate 600 python scripts/host_rate.py
exit 0
