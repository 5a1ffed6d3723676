#!/bin/bash
# rocprofv3 kernel-trace + stats of the graph-replayed bench step (short run, no side legs), the
# step list (tools/steplist.py) and the in-step family rooflines (tools/instep.py, aligned with
# the step's C-ABI calls from bench.py --dump-calls).
# Usage (on the GPU box): bash tools/profile.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-prof}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
  python3 $R/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-config5 --no-sliding --no-grouped --no-bf16 --no-dropin --no-data --no-exchange --dump-calls $OUT/calls.json "$@" > $OUT/bench.log 2>&1
rc=$?
echo "rocprofv3 rc=$rc"
[ $rc -eq 0 ] || exit $rc
KT=$(find $OUT -name "*kernel_trace.csv" | head -1)
python3 $R/tools/steplist.py $KT > $OUT/steplist.txt && tail -1 $OUT/steplist.txt
python3 $R/tools/instep.py $KT $OUT/calls.json $OUT/instep.json "${L3U_COMMIT:-}" "$*"
