#!/bin/bash
# sblock tests, stage timestamps, then the step A/B against L3U_SBLOCK=0
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sblock_gpu.py -q -x --timeout 120 --timeout-method thread -rf > gpurun_out/sb_test.log 2>&1
rc=$?; echo "sblock tests rc=$rc"; tail -15 gpurun_out/sb_test.log
[ $rc -eq 0 ] || exit $rc
L3U_LIB=$GRAFT_REPO_ROOT/light-3d-unet-front_amd/lib/var_sbprof.so timeout -k 10 200 python tools/sbprof.py || exit $?
bash tools/ab_env.sh L3U_SBLOCK "1 0" 2
