#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel trace,
# variant A/B.  Every GPU step has its own time limit; any failure ends it.
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
for s in ${STEPS:-smoke pytest bench prof tune}; do
  case $s in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()";;
    pytest) step pytest_gpu 700 python -m pytest tests -m gpu -q -x;;
    bench) step bench 400 python bench.py;;
    prof) step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary;;
    tune) step tune 300 python tools/tune_fixed.py;;
  esac
done
echo DONE
