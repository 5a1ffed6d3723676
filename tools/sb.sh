#!/bin/bash
# sblock check: its own tests first (a barrier bug must not reach the whole suite), then quick.sh
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sblock_gpu.py -q -x --timeout 120 --timeout-method thread -rf > gpurun_out/sb_test.log 2>&1
rc=$?; echo "sblock tests rc=$rc"; tail -15 gpurun_out/sb_test.log
[ $rc -eq 0 ] || exit $rc
bash tools/quick.sh ${1:-sb}
