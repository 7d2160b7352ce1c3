#!/bin/bash
# Same-box A/B of study libraries (LIBS="product gpu_study/x.so ...") on
# tools/sec_time.py sets (WHICH, default c1_1056), each library ROUNDS times, interleaved.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
i=0
for r in $(seq ${ROUNDS:-2}); do
  for lib in ${LIBS:-product}; do
    i=$((i+1))
    if [ "$lib" = product ]; then unset JLCRC_STUDY_LIB; else export JLCRC_STUDY_LIB=$lib; fi
    timeout -k 10 300 python3 tools/sec_time.py 10 ${WHICH:-c1_1056} > gpurun_out/abl_$i.log 2>&1 || { tail -3 gpurun_out/abl_$i.log; exit 1; }
    python3 - "$lib" gpurun_out/abl_$i.log <<'PY'
import json, sys
for l in open(sys.argv[2]):
    if l.startswith("{") and "ms_per_step" in l:
        d = json.loads(l); print(sys.argv[1], d["config"][:44], d["ms_per_step"], d.get("records_ok"))
PY
  done
done
