#!/bin/bash
# bench.py over variant libraries: bash tools/bench_variants.sh var_a.so var_b.so ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
for l in "$@"; do
  out=$(L3U_LIB=$R/light-3d-unet-front_amd/lib/$l timeout -k 10 300 python $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline ${BV_ARGS} 2>&1 | grep '"metric"') || { echo "fail $l"; exit 1; }
  echo "$l $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["roofline"]["avg_launch_ms"], d["fwd_ms_per_patch"])')" | tee -a $R/gpurun_out/bv.log
done
