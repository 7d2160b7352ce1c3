cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 300 python tools/tune_fixed.py > gpurun_out/r1_tune.log 2>&1; echo tune rc=$?; cat gpurun_out/r1_tune.log | grep -v amdgpu.ids
rc=$?
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r1_pytest_gpu2.log 2>&1; echo pytest rc=$?; tail -15 gpurun_out/r1_pytest_gpu2.log
