#!/bin/bash
# PMC passes on one kernel (regex $1) of `python tools/diag/run.py <lib>` ; one counter group per pass.
# usage: tools/prof_pmc.sh <kernel-regex> <tag>
export TMPDIR=/tmp
re=$1; tag=$2
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --kernel-trace --pmc $grp --kernel-include-regex "$re" --output-format csv \
     -d gpurun_out/pmc_${tag}_$i -o run -- python3 tools/diag/run.py mh-spgemm_amd/mhspgemm ${MATRIX:-cant} > gpurun_out/pmc_${tag}_$i.log 2>&1 || exit $?
done <<'GROUPS'
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM
SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM_RD SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL GRBM_GUI_ACTIVE GRBM_COUNT
TCC_HIT_sum TCC_MISS_sum
TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum
TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum
GROUPS
