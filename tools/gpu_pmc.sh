#!/bin/bash
# PMC passes (one counter group per rocprofv3 run, --pmc only; never combined
# with trace domains) over tools/sustain.py; summary in gpurun_out/${TAG}_pmc.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-pmc}
export TMPDIR=/tmp
export KINDS=${KINDS:-"crc3 stream"} LAUNCHES=${LAUNCHES:-6}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_p$i -o p -- python3 ${DRIVER:-tools/sustain.py} > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i ($grp) failed rc=$?"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done <<< "${GROUPS_LIST:-GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT
SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM
SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY
TA_TA_BUSY_sum TD_TD_BUSY_sum
FETCH_SIZE
WRITE_SIZE
SQ_ACTIVE_INST_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_ANY}"
python3 tools/pmc_summary.py gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.json && cat gpurun_out/${TAG}_pmc.json
