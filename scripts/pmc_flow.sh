#!/bin/bash
# PMC passes on k_rx, C2 without and with a one-flow table (one batch per
# launch), each pass its own rocprofv3 run under its own time limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="--steps 40 --warmup 4 --no-cpu --no-timing --streams 1 --fuse 1"
pass() {  # name bench-extra counters...
  local name=$1 extra=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --kernel-include-regex k_rx -f csv -d "gpurun_out/pmc_$name" -o run -- python3 bench.py $B $extra > "gpurun_out/pmc_$name.log" 2>&1
  local rc=$?; echo "pmc_$name rc=$rc"; [ $rc -eq 0 ] || exit $rc
}
for v in base flow; do
  X=""; [ $v = flow ] && X="--flow-capacity 1"
  pass ${v}_fetch "$X" FETCH_SIZE
  pass ${v}_write "$X" WRITE_SIZE
  pass ${v}_ea "$X" TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum
  pass ${v}_sq1 "$X" SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_INSTS_LDS
  pass ${v}_sq2 "$X" SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_SMEM
done
exit 0
