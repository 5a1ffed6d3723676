#!/bin/bash
# HBM-side traffic of the dominant call from PMC counters, one counter per pass (the guide's
# recipe: FETCH_SIZE and WRITE_SIZE do not fit one pass; no trace domains besides kernel-trace).
# Usage (GPU box): bash tools/pmc.sh <tag>
set -o pipefail
TAG=${1:-pmc}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o run -- \
    python3 $R/tools/pmc_dw.py > $OUT/$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
find $OUT -name "*counter_collection.csv" | head
