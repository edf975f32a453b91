#!/bin/bash
# Build an A/B library variant: packet-rs_amd/lib/variants/NAME.so with extra -D flags.
# usage: scripts/build_variant.sh NAME "-DPKTGPU_X=0 ..."
set -e
NAME=$1; shift
HERE=$(cd "$(dirname "$0")/.." && pwd)/packet-rs_amd
make -s -C "$HERE" OBJDIR="$HERE/build/obj_$NAME" LIB="$HERE/lib/variants/$NAME.so" \
  HIPFLAGS="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function $*" "$HERE/lib/variants/$NAME.so"
