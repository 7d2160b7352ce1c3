#!/bin/bash
# gv4 per-round cost study: tools/gv4_probe_k.py legs for the product build and
# study variants (tools/libjlcrc_study.so, general_v4.hip VAR) on one box.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"; mkdir -p gpurun_out; export TMPDIR=/tmp
LEGS=implicit_1152,sorted_1152,shuffled_1152,log_1057,implicit_4224 timeout -k 10 150 python3 tools/gv4_probe_k.py > gpurun_out/v0.log 2>&1 && tail -1 gpurun_out/v0.log || exit 1
export LEGS=implicit_1152,log_1057,implicit_4224
for v in ${VARIANTS:-8 9 5 6 7}; do
  JLCRC_STUDY_LIB=tools/libjlcrc_study.so GV4_VARIANT=$v timeout -k 10 150 python3 tools/gv4_probe_k.py > gpurun_out/v$v.log 2>&1 || exit 1; echo "v$v"; tail -1 gpurun_out/v$v.log
done
