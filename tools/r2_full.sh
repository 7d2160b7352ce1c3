# Usage: TAG=r2xx bash tools/r2_full.sh — smoke, GPU tests, bench, rocprofv3 kernel stats of the
# bench (C2 kernel) and of the C3/C5 timings; every step time-limited, the first failure ends it.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2}
step() {  # step <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/${T}_${name}.log" | tail -3 | cut -c1-400
  [ $rc -eq 0 ] || { echo "FATAL rc=$rc in $name"; exit $rc; }
}
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step pytest 700 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread
step bench 500 python bench.py
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary
step secprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_secprof -o run -- python3 tools/sec_time.py 5 all
echo DONE
