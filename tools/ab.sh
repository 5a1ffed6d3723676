# GPU A/B of two library builds on one box: the model / op GPU tests on the in-tree library, then
# REPS interleaved headline-step timings of lib/var_<A>.so and lib/var_<B>.so.
#   bash tools/ab.sh A B [REPS] [TAG]      (builds: tools/mkvar.sh; A_ENV / B_ENV: extra
#   environment of each side, e.g. A_ENV="L3U_SKIP_ABI_CHECK=1" for a build of an older commit;
#   AB_ARGS: extra bench arguments, e.g. "--enc 32,64,128,256 --size 64 --steps 20" for config 5;
#   AB_TESTS=0 skips the tests)
cd ${GRAFT_REPO_ROOT:-.}
A=${1:-prev}; B=${2:-cur}; REPS=${3:-3}; TAG=${4:-ab}
mkdir -p gpurun_out
if [ "${AB_TESTS:-1}" != "0" ]; then
  timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py tests/test_ops_gpu.py -m gpu -x -q --timeout 250 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -2 gpurun_out/${TAG}_tests.log
  [ $rc -eq 0 ] || exit $rc
fi
run() {
  env $2 L3U_LIB=$PWD/light-3d-unet-front_amd/lib/var_$1.so timeout -k 10 300 python bench.py --steps 60 --warmup 10 \
      --no-cpu-baseline --no-config5 --no-sliding --no-grouped --no-bf16 --no-dropin --no-data --no-exchange $AB_ARGS 2>&1 | grep metric | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$1', d['value'], d['ms_per_step'])"
}
for i in $(seq $REPS); do
  run $A "$A_ENV" || exit 1
  run $B "$B_ENV" || exit 1
done
