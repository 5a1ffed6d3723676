cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_sliding_gpu.py tests/test_bf16_gpu.py -m gpu -q --timeout 200 --timeout-method thread -rf > gpurun_out/r2h_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -12 gpurun_out/r2h_tests.log
