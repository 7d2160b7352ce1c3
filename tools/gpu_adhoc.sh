cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/r1_pytest_gpu4.log 2>&1; rc=$?; echo pytest rc=$rc; tail -4 gpurun_out/r1_pytest_gpu4.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu > gpurun_out/r1_bench4.log 2>&1; echo bench rc=$?; grep -v amdgpu.ids gpurun_out/r1_bench4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['roofline']); print(d.get('secondary'))"
