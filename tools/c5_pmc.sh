#!/bin/bash
# PMC passes over the fused log kernel (tools/c5_time.py, one C5 set); one
# counter group per rocprofv3 run.  Usage: SET=c1|mixed TAG=... bash tools/c5_pmc.sh
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-c5pmc}
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 200 rocprofv3 --pmc $grp --kernel-include-regex logstream_kernel --output-format csv -d gpurun_out/${TAG}_p$i -o p -- python3 tools/c5_time.py 3 ${SET:-c1} > gpurun_out/${TAG}_p$i.log 2>&1 || { echo "pass $i ($grp) failed"; tail -5 gpurun_out/${TAG}_p$i.log; exit 1; }
done <<< "${GROUPS_LIST:-GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH
SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM}"
python3 tools/pmc_summary.py gpurun_out/${TAG}_p* > gpurun_out/${TAG}_pmc.json && cat gpurun_out/${TAG}_pmc.json
