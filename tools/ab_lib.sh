#!/bin/bash
# Build an A/B copy of libdsgan_hip.so in which the listed csrc sources are taken from git revision
# REV and every other object is the in-tree build's (ds-gan_amd/build/obj), so a micro-benchmark can
# time the two forms of the changed kernels in one GPU call (tools/*_micro.py --libs a.so,b.so).
#   bash tools/ab_lib.sh REV OUT.so file.hip [file.hip ...]
set -e
REPO=$(cd "$(dirname "$0")/.." && pwd)
REV=$1; OUT=$2; shift 2
TMP=$(mktemp -d)
mkdir -p "$TMP/csrc"
git -C "$REPO" archive "$REV" ds-gan_amd/csrc | tar -x -C "$TMP"
OBJS=()
for o in "$REPO"/ds-gan_amd/build/obj/*.o; do
  b=$(basename "$o" .o)
  keep=1
  for f in "$@"; do [ "$b" = "$f" ] && keep=0; done
  [ $keep = 1 ] && OBJS+=("$o")
done
for f in "$@"; do
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -Wno-unused-result -I"$TMP/ds-gan_amd/csrc" \
      -c "$TMP/ds-gan_amd/csrc/$f" -o "$TMP/$f.o" &
  OBJS+=("$TMP/$f.o")
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" "${OBJS[@]}"
rm -rf "$TMP"
echo "built $OUT ($REV: $*)"
