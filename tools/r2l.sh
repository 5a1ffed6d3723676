cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/r2l_gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/r2l_gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r2l_smoke.log 2>&1; echo "smoke rc=$?"; tail -2 gpurun_out/r2l_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r2l_bench.log 2>&1; echo "bench rc=$?"; tail -c 600 gpurun_out/r2l_bench.log
