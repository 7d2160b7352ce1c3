# Usage: TAG=r2xx bash tools/r2_c3.sh — gv4 GPU tests, C3 timing, rocprofv3 kernel split of C3
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
T=${TAG:-r2}
timeout -k 10 300 python -u -m pytest tests/test_gpu_gv4.py tests/test_gpu_parity.py tests/test_gpu_robust.py tests/test_gpu_pipeline.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?
tail -1 gpurun_out/${T}_pytest.log
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_pytest.log | head -20; exit $rc; }
timeout -k 10 200 python tools/sec_time.py 10 c3 > gpurun_out/${T}_sec.log 2>&1 || { tail -20 gpurun_out/${T}_sec.log; exit 1; }
grep -o '"ms_per_step": [0-9.]*' gpurun_out/${T}_sec.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${T}_prof -o run -- python3 tools/sec_time.py 5 c3 > gpurun_out/${T}_prof.log 2>&1 || { tail -20 gpurun_out/${T}_prof.log; exit 1; }
f=$(ls gpurun_out/${T}_prof/*kernel_stats.csv | head -1)
grep -E "gv4" "$f" | sed -E 's/\(.*\)"//' | cut -d, -f1-4
