#!/bin/bash
# Runs the GPU test files one after another; stops at the first crash-like exit (not a plain
# test failure, rc 1), as gpurun's rules require.
mkdir -p gpurun_out
for f in "$@"; do
  timeout -k 10 ${STEP_TIMEOUT:-500} python -m pytest -q -m gpu -rf --tb=short "$f" > gpurun_out/$(basename $f .py).log 2>&1
  rc=$?
  echo "$f rc=$rc"; tail -5 gpurun_out/$(basename $f .py).log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after rc=$rc"; exit $rc; fi
done
