# A/B of study builds on C3 (and C5): gv4 tests through each variant first, then timings
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  JLCRC_STUDY_LIB=tools/libjlcrc_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_gv4.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_${v}_pytest.log 2>&1 || { tail -5 gpurun_out/ab_${v}_pytest.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/ab_${v}_pytest.log)"
done
bash tools/ab_wo.sh "$@"
