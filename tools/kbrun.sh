cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out; rm -f gpurun_out/kb.log
export KB_SHAPES="4,16,48 4,32,48 4,32,24 4,16,24"
KB_ARGS="--which fwd,fwd1,fwd1s" bash tools/kb.sh var_pd2.so var_pd3.so var_pd4.so var_pd2.so var_pd3.so var_pd4.so > /dev/null && \
KB_ARGS="--which bwd,bwd1" bash tools/kb.sh var_pd2.so var_gpd2.so var_gpd3.so var_pd2.so var_gpd2.so var_gpd3.so
