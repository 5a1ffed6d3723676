cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2e_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2e_tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/profile.sh r2e_f32
