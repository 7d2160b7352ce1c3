# Usage: TAG=r2xx bash tools/r2_gpu.sh  — GPU tests, then the C3/C5 timings (no profiler)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python tools/sec_time.py 10 all > gpurun_out/${T}_sec.log 2>&1 || { tail -20 gpurun_out/${T}_sec.log; exit 1; }
grep config gpurun_out/${T}_sec.log | cut -c1-330
