# Evidence of one commit (GPU box): fp32 / bf16 / config-5 step profiles with in-step
# family rooflines, the dominant call's PMC traffic, the step's PMC traffic + MFMA-busy passes
# and config 5's step traffic.   L3U_COMMIT=<sha> bash tools/run_evidence.sh <tag>
cd $GRAFT_REPO_ROOT
T=${1:-r3u}
export L3U_COMMIT=${L3U_COMMIT:-unknown}
bash tools/profile.sh ${T}_f32 || exit 1
bash tools/profile.sh ${T}_bf16 --dtype bf16 || exit 1
bash tools/profile.sh ${T}_c5 --enc 32,64,128,256 --size 64 || exit 1
bash tools/pmc.sh ${T}_pmcdw && python3 tools/pmc_json.py gpurun_out/${T}_pmcdw gpurun_out/${T}_pmc_dw3_bwd.json || exit 1
bash tools/pmc_step.sh ${T}_pmcstep && bash tools/pmc_gemm.sh ${T}_pmcgemm && \
  python3 tools/pmc_launch_json.py gpurun_out/${T}_pmcstep gpurun_out/${T}_pmcgemm gpurun_out/${T}_pmc_step.json || exit 1
bash tools/pmc_step.sh ${T}_c5pmc --enc 32,64,128,256 --size 64 || exit 1
bash tools/pmc_sq_step.sh ${T}_sq || exit 1
echo evidence done
