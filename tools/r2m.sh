cd $GRAFT_REPO_ROOT
bash tools/profile.sh r2m_f32 && bash tools/profile.sh r2m_bf16 --dtype bf16
