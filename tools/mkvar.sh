#!/bin/bash
# builds a variant of the C-ABI library with extra defines:  bash tools/mkvar.sh NAME "-DX=1 ..."
# -> light-3d-unet-front_amd/lib/var_NAME.so  (for tools/kb.sh / tools/bench_variants.sh)
# SRC=<dir> builds from another checkout's csrc/ (e.g. a `git worktree` of an older commit)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/light-3d-unet-front_amd
B=/tmp/l3u_var_$1
mkdir -p $B
SRCD=${SRC:-$P/csrc}
INCD=${SRC:+$SRC/../../include}
for f in $SRCD/*.hip; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-pass-failed \
    -I$SRCD -I${INCD:-$R/include} $2 -c $f -o $B/$(basename $f .hip).o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $P/lib/var_$1.so $B/*.o
echo built $P/lib/var_$1.so
