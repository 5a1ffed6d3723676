#!/bin/bash
# MFMA-busy and SQ-busy counters for every launch of one eager training step (one pass per group,
# kernel-trace only), plus the list of counters the box's rocprofv3 offers.
# Usage (GPU box): bash tools/pmc_gemm.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-pmcgemm}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for grp in "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES" "GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-config5 --no-sliding \
    --no-grouped --no-bf16 --no-dropin --no-data --no-exchange "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
find $OUT -name "*counter_collection.csv" | head
