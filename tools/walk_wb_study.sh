set -o pipefail
mkdir -p gpurun_out; export TMPDIR=/tmp
for v in base nowb; do
  if [ $v = base ]; then unset JLCRC_STUDY_LIB; else export JLCRC_STUDY_LIB=tools/libjlcrc_$v.so; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wp_$v -o run -- python3 tools/c5_time.py 5 c1 device > gpurun_out/wp_$v.log 2>&1 || { tail -5 gpurun_out/wp_$v.log; exit 1; }
  echo "$v: $(grep -E 'lc_walk|lc_build' gpurun_out/wp_$v/run_kernel_stats.csv | sed -E 's/\(.*\)"//' | cut -d, -f1,4 | tr '\n' ' ')"
done
