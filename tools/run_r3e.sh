cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread -k "bitwise or golden" > gpurun_out/r3e_model.log 2>&1
rc=$?; echo "model rc=$rc"; tail -3 gpurun_out/r3e_model.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r3e_gputest.log 2>&1
rc=$?; echo "all rc=$rc"; tail -4 gpurun_out/r3e_gputest.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh L3U_FRONT_R1 "0 1" 3 > gpurun_out/r3e_ab.log 2>&1; cat gpurun_out/r3e_ab.log
