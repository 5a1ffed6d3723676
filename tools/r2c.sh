cd $GRAFT_REPO_ROOT
bash tools/pmc_step.sh r2c_pmcstep && bash tools/pmc_gemm.sh r2c_pmcgemm
