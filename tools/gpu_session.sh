#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel trace,
# PMC traffic passes, variant A/B.  Every GPU step has its own time limit; any
# failure ends it.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r1}
export TMPDIR=/tmp
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_${name}.log" | tail -6
  [ $rc -eq 0 ] || { echo "FATAL rc=$rc in $name"; exit $rc; }
}
for s in ${STEPS:-smoke pytest bench prof pmc tune}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    pytest) step pytest_gpu 700 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread;;
    bench) step bench 400 python bench.py;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary;;
    pmc) KINDS="crc${PMC_CHAINS:-7}" GROUPS_LIST="FETCH_SIZE
WRITE_SIZE
TCC_EA0_RDREQ_sum
GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD
SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM" TAG=${TAG} step pmc 600 bash tools/gpu_pmc.sh;;
    tune) echo "tune: removed in r2 (study builds: tools/build_study.sh)";;
  esac
done
echo DONE
