#!/bin/bash
# A/B of study builds (tools/build_study.sh) on one box: the device-resident
# secondaries (tools/sec_time.py) per library, ROUNDS times interleaved (boxes
# differ by up to 5 %: only same-box comparisons count), results under gpurun_out/.
# LIBS: "product" (jleveldb_amd/libjlcrc.so), a study name v (tools/libjlcrc_v.so;
# tools/libjlcrc_*.so is gpurun-ignored, so copy it elsewhere first) or a path.
# Usage: TAG=r3i LIBS="product s8r1 dir/x.so" WHICH=dbbench_131 STEPS=20 ROUNDS=2
#        [PRE_PYTEST="-k dense"] bash tools/ab_lib.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-ab}
STEPS=${STEPS:-20}
WHICH=${WHICH:-c5}
if [ -n "$PRE_PYTEST" ]; then
  timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu $PRE_PYTEST \
    > gpurun_out/${TAG}_pytest.log 2>&1 || { tail -20 gpurun_out/${TAG}_pytest.log; exit 1; }
  tail -1 gpurun_out/${TAG}_pytest.log
fi
for r in $(seq ${ROUNDS:-1}); do
  for v in $LIBS; do
    case $v in
      product) lib= ;;
      */*|*.so) lib=$v ;;
      *) lib=tools/libjlcrc_$v.so ;;
    esac
    n=$(basename "$v" .so)
    echo "== $n (round $r)"
    JLCRC_STUDY_LIB=$lib timeout -k 10 300 python -u tools/sec_time.py $STEPS $WHICH > gpurun_out/${TAG}_${n}_$r.log 2>&1 \
      || { tail -5 gpurun_out/${TAG}_${n}_$r.log; exit 1; }
    python3 - gpurun_out/${TAG}_${n}_$r.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l)
        print(" ", d["config"][:48], d.get("ms_per_step"), d.get("GiB_per_s"), d.get("records_ok", ""),
              d.get("async_events_equal_sync", ""))
PY
  done
done
