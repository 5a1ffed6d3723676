#!/bin/bash
# Quick GPU check: pytest -m gpu, then the headline step only (no side legs), then optional kbench.
# usage: bash tools/quick.sh TAG [kbench --which list]
cd $GRAFT_REPO_ROOT
tag=$1
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread -rf > gpurun_out/${tag}_gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/${tag}_gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 60 --warmup 10 --no-cpu-baseline --no-config5 --no-sliding \
  --no-grouped --no-bf16 --no-dropin --no-data > gpurun_out/${tag}_hb$i.log 2>&1 || exit $?
grep -o '"value": [0-9.]*, "unit[^,]*, "n_gpus[^,]*, "steps[^,]*, "warmup[^,]*, "ms_per_step": [0-9.]*' gpurun_out/${tag}_hb$i.log
done
if [ -n "$2" ]; then timeout -k 10 300 python tools/kbench.py --which $2 > gpurun_out/${tag}_kb.log 2>&1; cat gpurun_out/${tag}_kb.log; fi
