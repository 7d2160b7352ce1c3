# Usage: TAG=r2xx [K="pytest -k expr"] bash tools/r2_c5.sh — GPU log tests, C5 timings, rocprofv3 kernel split of C5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2}
K=${K:-log or fullsize}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "$K" > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -2 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
timeout -k 10 300 python tools/sec_time.py 10 ${WHICH:-c5} > gpurun_out/${T}_sec.log 2>&1 || { tail -20 gpurun_out/${T}_sec.log; exit 1; }
grep config gpurun_out/${T}_sec.log | cut -c1-330
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 tools/c5_time.py 5 c1 device > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
f=$(ls gpurun_out/${T}_prof/*kernel_stats.csv | head -1)
cut -d, -f1-4 "$f" | grep -E "lc_|gv4|Name" | cut -c1-160
