#!/bin/bash
# step launch list with the fused small-volume block, and the A/B against L3U_SBLOCK=0
cd $GRAFT_REPO_ROOT
bash tools/profile.sh ${1:-sbp} || exit $?
f=$(find gpurun_out/${1:-sbp} -name "*kernel_trace.csv" | head -1)
python tools/steplist.py $f > gpurun_out/${1:-sbp}_steplist.txt && grep -E "sblock|sum" gpurun_out/${1:-sbp}_steplist.txt
bash tools/ab_env.sh L3U_SBLOCK "1 0" 2
