cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_fast_trainer_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/r2d_fast.log 2>&1
echo "fast rc=$?"
timeout -k 10 500 python bench.py --steps 50 --warmup 10 > gpurun_out/r2d_bench.log 2>&1
echo "bench rc=$?"
