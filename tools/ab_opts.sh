#!/bin/bash
# A/B of engine options (jl_set_option) on one box: the device-resident
# secondaries (tools/sec_time.py) per option set, ROUNDS times interleaved
# (boxes differ by a few per cent: only same-box comparisons count).
# Usage: TAG=r6j OPTS="base: lanes16k:12=16384 lanes64k:12=65536" WHICH=random_0_200 STEPS=10 ROUNDS=2 bash tools/ab_opts.sh
# Each OPTS entry is label:option=value[,option=value...] (empty after the colon: defaults).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-abo}
for r in $(seq ${ROUNDS:-1}); do
  for e in $OPTS; do
    n=${e%%:*}
    o=${e#*:}
    echo "== $n (round $r) [$o]"
    JL_OPTS=$o timeout -k 10 300 python -u tools/sec_time.py ${STEPS:-10} ${WHICH:-c5} > gpurun_out/${TAG}_${n}_$r.log 2>&1 \
      || { tail -20 gpurun_out/${TAG}_${n}_$r.log; exit 1; }
    python3 -c 'import json,sys
for l in open(sys.argv[1]):
    if l.startswith("{"):
        d = json.loads(l); print("  ", str(d.get("config", ""))[:60], d.get("ms_per_step"), d.get("records_ok", ""))' gpurun_out/${TAG}_${n}_$r.log
  done
done
echo DONE
