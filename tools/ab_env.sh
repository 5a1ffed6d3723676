#!/bin/bash
# A/B of an engine env switch on the headline step: bash tools/ab_env.sh VAR "v1 v2" ROUNDS
VAR=$1; VALS=$2; R=${3:-3}
for i in $(seq $R); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-config5 \
      --no-sliding --no-grouped --no-bf16 --no-dropin --no-data --no-exchange 2>&1 | grep metric | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$VAR=$v', d['value'], d['ms_per_step'])" || exit 1
  done
done
