cd $GRAFT_REPO_ROOT; mkdir -p gpurun_out; export TMPDIR=/tmp
# PMC A/B of instruction-cache / TLB / issue counters on C3: the product vs OLD_LIB (a library built from an older tree)
G="SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH SQ_WAIT_INST_ANY
TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_PENDING_STALL_CYCLES_sum
SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_VALU"
TAG=pnew DRIVER="tools/sec_time.py 3 c3" GROUPS_LIST="$G" bash tools/gpu_pmc.sh > gpurun_out/pnew.out 2>&1 || { tail -5 gpurun_out/pnew.out; exit 1; }
JLCRC_STUDY_LIB=${OLD_LIB:-jleveldb_amd/libjlcrc_old.so} TAG=pold DRIVER="tools/sec_time.py 3 c3" GROUPS_LIST="$G" bash tools/gpu_pmc.sh > gpurun_out/pold.out 2>&1 || { tail -5 gpurun_out/pold.out; exit 1; }
python3 - <<'PY'
import json
for t in ("pnew","pold"):
    d=json.load(open(f"gpurun_out/{t}_pmc.json"))
    for k,v in d.items():
        if "crc_gv4_kernel<0" in k: print(t, {c: round(x) for c,x in v.items()})
PY
