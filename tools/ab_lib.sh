#!/bin/bash
# A/B of variant libraries on the headline step: bash tools/ab_lib.sh "lib1.so lib2.so" ROUNDS
# (AB_ARGS: extra bench arguments, e.g. the config-5 shape)
LIBS=$1; R=${2:-3}
cd ${GRAFT_REPO_ROOT:-.}
for i in $(seq $R); do
  for l in $LIBS; do
    L3U_LIB=$PWD/light-3d-unet-front_amd/lib/$l timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-config5 \
      --no-sliding --no-grouped --no-bf16 --no-dropin --no-data --no-exchange $AB_ARGS 2>&1 | grep metric | \
      python -c "import sys,json; d=json.loads(sys.stdin.read()); print('$l', d['value'], d['ms_per_step'])" || exit 1
  done
done
