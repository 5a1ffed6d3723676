cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py tests/test_bf16_gpu.py tests/test_model_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2f_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r2f_tests.log
[ $rc -eq 0 ] || exit $rc
rm -f gpurun_out/bv.log
BV_ARGS="--no-sliding --no-config5 --no-grouped --no-bf16 --no-dropin" bash tools/bench_variants.sh libl3u_hip.so var_ks128.so libl3u_hip.so var_ks128.so
