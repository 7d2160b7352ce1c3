set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r2t_pytest.log 2>&1; rc=$?
tail -25 gpurun_out/r2t_pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/c5_time.py 10 both device > gpurun_out/r2t_c5.log 2>&1 || { tail -20 gpurun_out/r2t_c5.log; exit 1; }
cat gpurun_out/r2t_c5.log | grep -v amdgpu.ids
