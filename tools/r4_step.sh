#!/bin/bash
# Round-4 GPU session: log parity tests first (the new dense-block kernel), then
# the whole GPU suite, the C5 / C3 timings, a kernel trace of the C5 sets, and
# the bench.  Each step under its own limit; the first failure ends the call.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r4}
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${T}_${name}.log" 2>&1; local rc=$?
  echo "   rc=$rc"; grep -v amdgpu.ids "gpurun_out/${T}_${name}.log" | tail -${TAIL:-4} | cut -c1-400
  [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "gpurun_out/${T}_${name}.log" | head -20; echo "FATAL rc=$rc in $name"; exit $rc; }
}
for s in ${STEPS:-logtests pytest sec bench}; do
  case $s in
    logtests) run logtests 300 python -u -m pytest tests/test_gpu_logstream.py tests/test_gpu_log_shapes.py -m gpu -x -q --timeout 120 --timeout-method thread;;
    pytest) run pytest 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${K:+-k "$K"};;
    sec) run sec 400 python3 tools/sec_time.py 10 ${WHICH:-all};;
    secprof) run secprof 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_secprof -o run -- python3 tools/sec_time.py 5 ${WHICH:-c5};;
    bench) run bench 600 python bench.py;;
    prof) run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-secondary;;
    *) echo "unknown step $s"; exit 2;;
  esac
done
echo DONE
