#!/bin/bash
# bench + rocprofv3 kernel trace + PMC passes (separate runs, per the guide).
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
TAG=${TAG:-r1}
set -o pipefail
step() { local name=$1 t=$2; shift 2; echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1; local rc=$?; echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/${TAG}_${name}.log" | tail -4; [ $rc -eq 0 ] || exit $rc; }
step bench 400 python bench.py
export TMPDIR=/tmp
step prof_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o trace -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary
step prof_fetch 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_prof -o pmc_fetch -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary
step prof_write 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${TAG}_prof -o pmc_write -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary
step prof_tcc 300 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d gpurun_out/${TAG}_prof -o pmc_rdreq -- python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary
echo DONE
