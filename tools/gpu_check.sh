#!/bin/bash
# One GPU session: smoke, GPU parity tests, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault/abort/timeout ends the script.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-r1}
fatal() { case "$1" in 0|1) return 1;; *) echo "FATAL rc=$1 in $2"; exit "$1";; esac; }
run() {  # run <name> <timeout> cmd...
  local name=$1 t=$2; shift 2
  echo "== $name"; timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1; local rc=$?
  echo "   rc=$rc"; tail -5 "gpurun_out/${TAG}_${name}.log"
  fatal $rc "$name" || true
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run pytest_gpu 700 python -m pytest tests -m gpu -q -x
run bench 400 python bench.py
cd /tmp && export TMPDIR=/tmp && cd "$OLDPWD"
run rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu --no-secondary
echo DONE
