#!/bin/bash
# Same-box A/B of study variants of crc_gv4_kernel (tools/libjlcrc_study.so,
# general_v4.hip VAR) against the product, interleaved: VARIANTS="0 2 0 2"
# (0 = the product library), WHICH = tools/sec_time.py sets (default c3).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for v in ${VARIANTS:-0 2 0 2}; do
  i=$((i+1))
  if [ "$v" = 0 ]; then unset JLCRC_STUDY_LIB GV4_VARIANT; else export JLCRC_STUDY_LIB=tools/libjlcrc_study.so GV4_VARIANT=$v; fi
  timeout -k 10 300 python3 tools/sec_time.py 10 ${WHICH:-c3} > gpurun_out/abv_$i.log 2>&1 || { tail -3 gpurun_out/abv_$i.log; exit 1; }
  python3 - "$v" gpurun_out/abv_$i.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{") and "ms_per_step" in l:
        d = json.loads(l); print("variant", sys.argv[1], d["config"][:44], d["ms_per_step"])
PY
done
