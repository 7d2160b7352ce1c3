# PMC passes (one group per run) over the C3 gv4 launch (tools/c3_driver.py) and the
# C2 4 KiB kernel (bench.py), same counter groups; summaries in gpurun_out/${TAG}_{c3,c2}_pmc.json
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out && export TMPDIR=/tmp
T=${TAG:-r2p}
G="GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_ANY
SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INST_LEVEL_VMEM SQ_WAVE_CYCLES SQ_INSTS_BRANCH SQ_WAIT_ANY SQ_WAIT_INST_LDS
TA_TA_BUSY_sum TD_TD_BUSY_sum TCP_TCC_READ_REQ_sum"
for w in c3 c2; do
  i=0
  while read -r grp; do
    i=$((i+1))
    if [ $w = c3 ]; then cmd="python3 tools/c3_driver.py"; else cmd="python3 bench.py --steps 3 --warmup 1 --no-cpu --no-secondary"; fi
    C3_PATH=gv4 LAUNCHES=3 timeout -k 10 150 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${T}_${w}_p$i -o p -- $cmd > gpurun_out/${T}_${w}_p$i.log 2>&1 || { echo "$w pass $i failed"; tail -5 gpurun_out/${T}_${w}_p$i.log; exit 1; }
  done <<< "$G"
  python3 tools/pmc_summary.py gpurun_out/${T}_${w}_p* > gpurun_out/${T}_${w}_pmc.json || exit 1
done
python3 - <<'PY'
import json, os
T = os.environ.get("TAG", "r2p")
for w, k in (("c3", "crc_gv4_kernel<0, 0>"), ("c2", "crc_fixed4k_v4_kernel")):
    d = json.load(open(f"gpurun_out/{T}_{w}_pmc.json"))
    for name, v in d.items():
        if k in name:
            print(w, json.dumps({c: v[c] for c in sorted(v)}))
PY
