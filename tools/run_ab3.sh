cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
run() {  # lib r1
  L3U_LIB=$PWD/light-3d-unet-front_amd/lib/$1 L3U_FRONT_R1=$2 timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-config5 \
      --no-sliding --no-grouped --no-bf16 --no-dropin --no-data 2>&1 | grep metric | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$1 R1=$2', d['value'], d['ms_per_step'])"
}
for i in 1 2 3; do
  run var_prev.so 0 || exit 1
  run var_cur.so 0 || exit 1
  run var_cur.so 1 || exit 1
done
