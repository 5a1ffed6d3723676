#!/bin/bash
# rocprofv3 kernel-trace + stats of the default bench workload (short run, no CPU baseline).
# Usage (on the GPU box): bash tools/profile.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-prof}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config5 --no-sliding --no-grouped --no-bf16 --no-dropin --no-data "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
find $OUT -name "*kernel_stats.csv" | head -3
exit $rc
