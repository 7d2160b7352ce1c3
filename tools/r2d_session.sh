set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 400 --timeout-method thread > gpurun_out/r2d_fullsize.log 2>&1 || { tail -30 gpurun_out/r2d_fullsize.log; exit 1; }
tail -8 gpurun_out/r2d_fullsize.log
timeout -k 10 400 python bench.py > gpurun_out/r2d_bench.log 2>&1 || { tail -20 gpurun_out/r2d_bench.log; exit 1; }
tail -c 3000 gpurun_out/r2d_bench.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r2d_prof -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu > gpurun_out/r2d_prof.log 2>&1 || { tail -20 gpurun_out/r2d_prof.log; exit 1; }
echo PROF_OK
