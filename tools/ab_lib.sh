#!/bin/bash
# A/B of study builds (tools/build_study.sh) on one box: the device-resident
# secondaries (tools/sec_time.py) once per library, results under gpurun_out/.
# Usage: TAG=r3i LIBS="s4r2 s8r1" WHICH=dbbench_131 STEPS=20 [PRE_PYTEST="-k dense"] bash tools/ab_lib.sh
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
TAG=${TAG:-ab}
STEPS=${STEPS:-20}
WHICH=${WHICH:-c5}
if [ -n "$PRE_PYTEST" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $PRE_PYTEST \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
fi
for v in $LIBS; do
  lib=tools/libjlcrc_$v.so
  [ "$v" = product ] && lib=
  echo "== $v"
  JLCRC_STUDY_LIB=$lib timeout -k 10 300 python -u tools/sec_time.py $STEPS $WHICH > gpurun_out/${TAG}_$v.log 2>&1 \
    || { tail -5 gpurun_out/${TAG}_$v.log; exit 1; }
  python3 - gpurun_out/${TAG}_$v.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(" ", d["config"][:48], d.get("ms_per_step"), d.get("GiB_per_s"), d.get("records_ok", ""),
              d.get("async_events_equal_sync", ""))
PY
done
