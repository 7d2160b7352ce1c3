# C3 footprint study: gv4 / stream kernel time and the read ceiling at 1/4, 1/2, 1x of C3
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
for nb in 262144 524288 1048576; do
  for g in stream gv4; do
    C3_N=$nb C3_STREAM=1 C3_PATH=$g LAUNCHES=6 timeout -k 10 120 python3 tools/c3_driver.py 2>&1 | grep -v amdgpu.ids || exit 1
  done
done
