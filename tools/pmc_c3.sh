# PMC passes over tools/c3_driver.py (C3 through the general path); TAG / C3_PATH from the env
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && export TMPDIR=/tmp
g=${C3_PATH:-gv4}
C3_PATH=$g timeout -k 10 120 python3 tools/c3_driver.py > gpurun_out/${TAG}_$g.log 2>&1 || exit 1
C3_PATH=$g DRIVER=tools/c3_driver.py TAG=${TAG}_$g GROUPS_LIST="FETCH_SIZE
GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_ANY
TA_TA_BUSY_sum TD_TD_BUSY_sum" LAUNCHES=3 bash tools/gpu_pmc.sh > gpurun_out/${TAG}_${g}_pmcrun.log 2>&1 || exit 1
echo ok
