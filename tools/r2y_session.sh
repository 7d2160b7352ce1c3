set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2y_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r2y_pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/r2y_pytest.log | head -20; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2y_prof -o run -- python3 tools/c5_time.py 5 c1 device > gpurun_out/r2y_prof.log 2>&1 || { tail -20 gpurun_out/r2y_prof.log; exit 1; }
grep config gpurun_out/r2y_prof.log | cut -c1-300
i=0
while read -r grp; do
  i=$((i+1))
  timeout -k 10 120 rocprofv3 --pmc $grp --kernel-include-regex "gv4_kernel|lc_" --output-format csv -d gpurun_out/r2y_p$i -o p -- python3 tools/c5_time.py 2 c1 device > gpurun_out/r2y_p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/r2y_p$i.log; exit 1; }
done <<< "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH
SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU
SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INST_LEVEL_VMEM"
python3 tools/pmc_summary.py gpurun_out/r2y_p* > gpurun_out/r2y_pmc.json && cat gpurun_out/r2y_pmc.json
