#!/bin/bash
# PMC passes over the kernel microbench (scripts/kvariants). Continues past a
# pass that fails to configure (unknown counter), stops on fault/timeout.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out; export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || rocprofv3 --list-avail > gpurun_out/pmc_list.txt 2>&1
grep -o "SQ_[A-Z_0-9]*\|TCC_EA0_[A-Z_0-9]*\|TCP_[A-Z_0-9]*\|GRBM_[A-Z_0-9]*" gpurun_out/pmc_list.txt | sort -u > gpurun_out/pmc_names.txt
i=0
while read -r set; do
  i=$((i+1))
  timeout -k 10 180 rocprofv3 --pmc $set --kernel-include-regex "k_rx|k_glds" -f csv -d gpurun_out/pmc_$i -o run -- ./scripts/kvariants 40 > gpurun_out/pmc_$i.log 2>&1
  rc=$?; echo "pass $i ($set) rc=$rc"
  if [ $rc -eq 124 ] || [ $rc -eq 134 ] || [ $rc -eq 137 ] || [ $rc -eq 139 ]; then exit $rc; fi
done <<'SETS'
SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE
SQ_INSTS_BRANCH SQ_ACTIVE_INST_SALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS SQ_BUSY_CYCLES
SETS
exit 0
