# GPU-test the tree, then the fp32 and config-5 step profiles and config-5 PMC step traffic.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export L3U_COMMIT=${L3U_COMMIT:-unknown}
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r3g_gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3g_gputest.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh r3g_f32 && bash tools/profile.sh r3g_c5 --enc 32,64,128,256 --size 64 && \
  bash tools/pmc_step.sh r3g_c5pmc --enc 32,64,128,256 --size 64
