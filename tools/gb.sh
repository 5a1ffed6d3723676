#!/bin/bash
# GEMM microbench over variant libraries: bash tools/gb.sh lib1.so lib2.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for l in "$@"; do
  L3U_LIB=$R/light-3d-unet-front_amd/lib/$l timeout -k 10 300 python $R/tools/gemmbench.py >> $R/gpurun_out/gb.log 2>&1 || { echo "fail $l rc=$?"; exit 1; }
done
grep -v amdgpu.ids $R/gpurun_out/gb.log
