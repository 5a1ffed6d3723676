#!/bin/bash
# SQ counters (waves, VALU / SALU / VMEM / LDS instruction counts, wait and busy cycles) of every
# launch of one eager training step: two passes of <= 8 SQ counters, kernel-trace only (the
# MI355X_MICROARCH.md recipe), then tools/sq_step_json.py -> one record per launch.
# Usage (GPU box): bash tools/pmc_sq_step.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-sqstep}; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd /tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- \
    python3 $R/bench.py --steps 2 --warmup 1 --no-graph --no-cpu-baseline --no-config5 --no-sliding \
    --no-grouped --no-bf16 --no-dropin --no-data --no-exchange "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 $R/tools/sq_step_json.py $OUT $OUT/sq_step.json
