cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_bf16_gpu.py -k "oracle" -m gpu -x -v -s --timeout 250 --timeout-method thread > gpurun_out/r3d_bf16.log 2>&1
echo "bf16 rc=$?"; grep -E "vs bf16-storage|passed|failed|Error" gpurun_out/r3d_bf16.log | tail -8
timeout -k 10 200 python tools/pwbench.py --scale --iters 20 > gpurun_out/pwscale.log 2>&1
echo "pw rc=$?"; tail -22 gpurun_out/pwscale.log
