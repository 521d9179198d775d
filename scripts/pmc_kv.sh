#!/bin/bash
# PMC passes on the kernel microbench; continue past unconfigurable passes.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
TAG=${TAG:-kv}
i=0
while read -r set; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-include-regex "k_rx|k_glds" -f csv -d gpurun_out/${TAG}_$i -o run -- ./scripts/kvariants 40 > gpurun_out/${TAG}_$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
done <<'SETS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
FETCH_SIZE
WRITE_SIZE
SETS
exit 0
