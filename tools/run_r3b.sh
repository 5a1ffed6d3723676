cd $GRAFT_REPO_ROOT
export L3U_COMMIT=56170eb
bash tools/profile.sh r3b_f32 && bash tools/profile.sh r3b_c5 --enc 32,64,128,256 --size 64 && bash tools/pmc_step.sh r3b_c5pmc --enc 32,64,128,256 --size 64
