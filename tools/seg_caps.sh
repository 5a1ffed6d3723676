#!/bin/bash
# step time over reduction-item caps: bash tools/seg_caps.sh "32,16,8" "64,32,16" ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
for c in "$@"; do
  out=$(L3U_SEG_CAPS=$c timeout -k 10 300 python $R/bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-config5 --no-sliding --no-grouped 2>&1 | grep '"metric"') || { echo "fail $c"; exit 1; }
  echo "$c $(echo "$out" | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
