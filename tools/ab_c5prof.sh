# C5 kernel split (both payload sets) per study variant: rocprofv3 kernel trace of tools/sec_time.py c5
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in base "$@"; do
  if [ $v = base ]; then unset JLCRC_STUDY_LIB; else export JLCRC_STUDY_LIB=tools/libjlcrc_$v.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/abp_$v -o run -- python3 tools/sec_time.py 5 c5 > gpurun_out/abp_$v.log 2>&1 || { tail -5 gpurun_out/abp_$v.log; exit 1; }
  echo "$v: $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abp_$v.log | tr '\n' ' ')"
  grep -E "lc_|gv4" gpurun_out/abp_$v/run_kernel_stats.csv | sed -E 's/\(.*\)"//' | cut -d, -f1,2,4 | tr '\n' ' '; echo
done
