#!/bin/bash
# Full GPU check: pytest -m gpu, smoke(), bench.py; stops at the first crash-like exit.
# usage: bash tools/full.sh TAG [bench args...]
cd $GRAFT_REPO_ROOT
tag=$1; shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rf > gpurun_out/${tag}_gputest.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -5 gpurun_out/${tag}_gputest.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1; rc=$?; echo "smoke rc=$rc"; tail -2 gpurun_out/${tag}_smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py "$@" > gpurun_out/${tag}_bench.log 2>&1; echo "bench rc=$?"; tail -c 1500 gpurun_out/${tag}_bench.log
