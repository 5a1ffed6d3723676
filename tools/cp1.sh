#!/bin/bash
# convT pair-fusion check: op + model tests, then the A/B of the fused launch
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_model_gpu.py tests/test_bf16_gpu.py -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/cp1_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/cp1_test.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh "libl3u_hip.so var_nopair1.so" 3
