#!/bin/bash
# vectorized AdamW tick: model / trainer tests, then the A/B against the previous library
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py tests/test_bf16_gpu.py -q -x --timeout 200 --timeout-method thread -rf > gpurun_out/aw_test.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 gpurun_out/aw_test.log
[ $rc -eq 0 ] || exit $rc
bash tools/ab_lib.sh "libl3u_hip.so var_head.so" 3
