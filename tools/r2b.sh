cd $GRAFT_REPO_ROOT
bash tools/profile.sh r2b_f32 && bash tools/profile.sh r2b_bf16 --dtype bf16
