#!/bin/bash
# pw backward microbench over variant libraries: bash tools/pwb.sh lib1.so lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for l in "$@"; do
  L3U_LIB=$R/light-3d-unet-front_amd/lib/$l timeout -k 10 300 python $R/tools/pwbench.py >> $R/gpurun_out/pwb.log 2>&1 || { echo "fail $l rc=$?"; exit 1; }
done
grep -v amdgpu.ids $R/gpurun_out/pwb.log
