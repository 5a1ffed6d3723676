cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/r2a_gputest.log 2>&1 && \
timeout -k 10 400 python bench.py --steps 50 --warmup 10 > gpurun_out/r2a_bench.log 2>&1 && \
timeout -k 10 300 python bench.py --dtype bf16 --steps 50 --warmup 10 --no-cpu-baseline --no-sliding --no-config5 --no-grouped > gpurun_out/r2a_bench_bf16.log 2>&1
echo rc=$?
