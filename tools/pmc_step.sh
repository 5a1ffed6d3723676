#!/bin/bash
# HBM-side traffic of every kernel of the eager training step (FETCH_SIZE and WRITE_SIZE in
# separate passes, kernel-trace only, as MI355X_MICROARCH.md prescribes).
# Usage (GPU box): bash tools/pmc_step.sh <tag> [extra bench args, e.g. --enc 32,64,128,256 --size 64]
set -o pipefail
TAG=${1:-pmcstep}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 240 rocprofv3 --pmc $c --kernel-trace --output-format csv -d $OUT/$c -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-config5 --no-sliding \
    --no-grouped --no-bf16 --no-dropin --no-data --no-exchange "$@" > $OUT/$c.log 2>&1 || { echo "pass $c failed"; exit 1; }
done
python3 $R/tools/pmc_step_json.py $OUT $OUT/pmc_step.json
