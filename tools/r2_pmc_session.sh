#!/bin/bash
# r2 traffic passes: FETCH_SIZE / WRITE_SIZE (/ TCC_EA0_RDREQ_sum) per launch of
# the C2 4 KiB kernel, the C3 general v4 kernel and the C5 two-pass kernels; one
# counter per rocprofv3 --pmc run (tools/gpu_pmc.sh).  Summaries in
# gpurun_out/${TAG}_{fx,c3,c5c1,c5mx}_pmc.json.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r2r}
set -o pipefail
KINDS=crc7 TAG=${TAG}_fx GROUPS_LIST="FETCH_SIZE
WRITE_SIZE
TCC_EA0_RDREQ_sum" bash tools/gpu_pmc.sh > gpurun_out/${TAG}_fx_run.log 2>&1 || { echo "fx failed"; tail gpurun_out/${TAG}_fx_run.log; exit 1; }
C3_PATH=gv4 DRIVER=tools/c3_driver.py LAUNCHES=3 TAG=${TAG}_c3 GROUPS_LIST="FETCH_SIZE
WRITE_SIZE" bash tools/gpu_pmc.sh > gpurun_out/${TAG}_c3_run.log 2>&1 || { echo "c3 failed"; tail gpurun_out/${TAG}_c3_run.log; exit 1; }
for s in c1 mixed; do
  i=0
  for grp in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_c5${s}_p$i -o p -- python3 tools/c5_time.py 3 $s device > gpurun_out/${TAG}_c5${s}_p$i.log 2>&1 || { echo "c5 $s $grp failed"; tail gpurun_out/${TAG}_c5${s}_p$i.log; exit 1; }
  done
  python3 tools/pmc_summary.py gpurun_out/${TAG}_c5${s}_p* > gpurun_out/${TAG}_c5${s}_pmc.json
done
echo done
