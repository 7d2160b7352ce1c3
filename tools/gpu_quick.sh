#!/bin/bash
# Quick GPU check: the log-shape tests first, then the GPU suite, then C3 / C5 timings.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
T=${TAG:-g6}
timeout -k 10 300 python -u -m pytest tests/test_gpu_log_shapes.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_shapes.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_shapes.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_shapes.log | head -20; exit $rc; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_pytest.log 2>&1; rc=$?; tail -1 gpurun_out/${T}_pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" gpurun_out/${T}_pytest.log | head -30; exit $rc; }
timeout -k 10 400 python3 tools/sec_time.py 10 all > gpurun_out/${T}_sec.log 2>&1 && grep -v amdgpu gpurun_out/${T}_sec.log | cut -c1-300
