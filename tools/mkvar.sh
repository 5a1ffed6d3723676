#!/bin/bash
# builds a variant of the C-ABI library with extra defines:  bash tools/mkvar.sh NAME "-DX=1 ..."
# -> light-3d-unet-front_amd/lib/var_NAME.so  (for tools/kb.sh / tools/bench_variants.sh / tools/ab.sh)
# SRC=<dir> builds from another checkout's csrc/ (e.g. a `git worktree` of an older commit)
# ONLY="dwconv misc" compiles just those sources with the defines and links the other objects of
# the in-tree build (light-3d-unet-front_amd/build/*.o: run `make` first)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
P=$R/light-3d-unet-front_amd
B=/tmp/l3u_var_$1
rm -rf $B
mkdir -p $B
SRCD=${SRC:-$P/csrc}
INCD=${SRC:+$SRC/../../include}
for f in $SRCD/*.hip; do
  b=$(basename $f .hip)
  if [ -n "$ONLY" ] && ! echo " $ONLY " | grep -q " $b "; then
    cp $P/build/$b.o $B/$b.o
    continue
  fi
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-pass-failed \
    -I$SRCD -I${INCD:-$R/include} $2 -c $f -o $B/$b.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $B/var.so $B/*.o && mv -f $B/var.so $P/lib/var_$1.so
echo built $P/lib/var_$1.so
