# The driver's own round-end commands on one tree (GPU box), logs under gpurun_out/<tag>_final_*:
#   bash tools/run_final.sh <sha> [tag]
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
SHA=${1:-unknown}
T=${2:-r4}
echo "commit $SHA" > gpurun_out/${T}_final_gputest.log
timeout -k 10 900 python -m pytest tests -x -q -m gpu >> gpurun_out/${T}_final_gputest.log 2>&1
rc=$?; echo "gputest rc=$rc"; tail -2 gpurun_out/${T}_final_gputest.log; [ $rc -eq 0 ] || exit $rc
echo "commit $SHA" > gpurun_out/${T}_final_smoke.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" >> gpurun_out/${T}_final_smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/${T}_final_smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${T}_final_bench.json 2> gpurun_out/${T}_final_bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 gpurun_out/${T}_final_bench.json; exit $rc
