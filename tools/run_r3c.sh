cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_device_loader_gpu.py tests/test_lesion_gpu.py tests/test_bench_launch_gpu.py tests/test_patches_gpu.py -m gpu -x -v --timeout 500 --timeout-method thread > gpurun_out/r3c_new.log 2>&1
rc=$?; echo "new rc=$rc"; tail -15 gpurun_out/r3c_new.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r3c_gputest.log 2>&1
rc=$?; echo "all rc=$rc"; tail -5 gpurun_out/r3c_gputest.log
