#!/bin/bash
# Link an alternative pagerank.hip (measurement experiments) against the other
# objects of the current build: scripts/build_variant.sh <variant.hip> <out.so>
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$ROOT/cugraph-forked_amd"
OBJ=$(mktemp /tmp/variant.XXXXXX.o)
/opt/rocm/bin/hipcc -std=c++17 -O3 -fPIC --offload-arch=gfx950 -I"$PKG/../include" -I"$PKG/csrc" -Wno-unused-result ${VARIANT_FLAGS:-} \
  -x hip -c "$1" -o "$OBJ"
OTHERS=$(ls "$PKG"/build/*.o | grep -v "/$(basename $1).o$")
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o "$2" $OBJ $OTHERS
rm -f "$OBJ"
