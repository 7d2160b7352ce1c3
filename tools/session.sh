#!/bin/bash
# One parameterised GPU session (replaces the per-session r2*/ab_* scripts).
#   TAG=r3a STEPS="smoke pytest bench prof secprof" [K="pytest -k expr"] [PYTEST_PATHS="tests/x.py ..."]
#   [SETS="c1_1056 dbbench_131"] bash tools/session.sh
# Steps (each under its own time limit; the first failure ends the session):
#   smoke    __graft_entry__.smoke()
#   pytest   the GPU tests (-m gpu, optionally -k "$K" / PYTEST_PATHS)
#   bench    python bench.py (the driver's default command)
#   prof     rocprofv3 kernel stats of the C2 bench (roofline kernel)
#   secprof  rocprofv3 kernel stats of the C3 and C5 secondaries (tools/sec_time.py)
#   sec      C3 / C5 timings without the profiler (tools/sec_time.py)
#   pmc      traffic passes FETCH_SIZE / WRITE_SIZE (one counter per rocprofv3 run) over
#            tools/sec_time.py $PMC_WHICH ($PMC_KERNEL filters the kernels)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r3}
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/${T}_${name}.log" | tail -${TAIL:-4} | cut -c1-600
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "gpurun_out/${T}_${name}.log" | head -20; echo "FATAL rc=$rc in $name"; exit $rc; }
}
for s in ${STEPS:-smoke pytest bench}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    pytest) step pytest 900 python -u -m pytest ${PYTEST_PATHS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread ${K:+-k "$K"};;
    bench) step bench 600 python bench.py;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary;;
    sec) step sec 400 python3 tools/sec_time.py 10 ${WHICH:-all};;
    secprof) step secprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_secprof -o run -- python3 tools/sec_time.py 5 ${WHICH:-all};;
    pmc) i=0
         for grp in FETCH_SIZE WRITE_SIZE ${PMC_EXTRA}; do
           i=$((i+1))
           step pmc_p$i 240 rocprofv3 --pmc $grp ${PMC_KERNEL:+--kernel-include-regex "$PMC_KERNEL"} --output-format csv -d gpurun_out/${T}_pmc_p$i -o p -- python3 tools/sec_time.py 3 ${PMC_WHICH:-c5}
         done
         python3 tools/pmc_summary.py gpurun_out/${T}_pmc_p* > gpurun_out/${T}_pmc.json && head -c 1500 gpurun_out/${T}_pmc.json;;
    *) echo "unknown step $s"; exit 2;;
  esac
done
echo DONE
