#!/bin/bash
# A/B/C of env settings on the headline step: bash tools/ab_env2.sh ROUNDS "A=1 B=0" "A=1 B=1" ...
R=$1; shift
for i in $(seq $R); do
  for cfg in "$@"; do
    env $cfg timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-config5 \
      --no-sliding --no-grouped --no-bf16 --no-dropin --no-data 2>&1 | grep metric | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('[$cfg]', d['value'], d['ms_per_step'])" || exit 1
  done
done
