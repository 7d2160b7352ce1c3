#!/bin/bash
# Same-box A/B of the product library against jleveldb_amd/libjlcrc_old.so
# (C3 and the C5 sets through tools/sec_time.py), interleaved twice.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for i in 1 2; do
  for lib in new old; do
    if [ $lib = old ]; then export JLCRC_STUDY_LIB=jleveldb_amd/libjlcrc_old.so; else unset JLCRC_STUDY_LIB; fi
    timeout -k 10 300 python3 tools/sec_time.py 10 ${WHICH:-c3,c1_1056,mixed_1b_100k} > gpurun_out/ab_$lib$i.log 2>&1 || { tail -3 gpurun_out/ab_$lib$i.log; exit 1; }
    python3 -c "
import json,sys
for l in open('gpurun_out/ab_$lib$i.log'):
    if l.startswith('{') and 'ms_per_step' in l:
        d=json.loads(l); print('$lib$i', d['config'][:40], d['ms_per_step'])"
  done
done
