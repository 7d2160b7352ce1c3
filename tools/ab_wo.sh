# A/B timings of study builds against the product library: bash tools/ab_wo.sh <variant>...
set -o pipefail
mkdir -p gpurun_out
for i in 1 2; do
for v in base "$@"; do
  if [ $v = base ]; then unset JLCRC_STUDY_LIB; else export JLCRC_STUDY_LIB=tools/libjlcrc_$v.so; fi
  timeout -k 10 200 python tools/sec_time.py 10 all > gpurun_out/ab_${v}_$i.log 2>&1 || { tail -5 gpurun_out/ab_${v}_$i.log; exit 1; }
  echo "$v $i $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${v}_$i.log | tr '\n' ' ')"
done; done
