#!/bin/bash
# build an experimental libgossip_hip.so variant: build_variant.sh NAME "-DFLAG=..."
# output: gossip-protocol-with-power-law_amd/_ab/NAME.so (git-ignored, travels to the GPU box)
set -e
cd "$(dirname "$0")/.."
PKG=gossip-protocol-with-power-law_amd
OUT=$PKG/_ab/$1
mkdir -p $OUT
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 $2"
SRCS=$(python3 -c "import sys; sys.path.insert(0, '$PKG'); import build_lib; print(' '.join(build_lib.SOURCES))")
for s in $SRCS; do
  /opt/rocm/bin/hipcc $F -c $PKG/csrc/$s -o $OUT/${s%.hip}.o &
done
wait
/opt/rocm/bin/hipcc $F -shared $OUT/*.o -o $PKG/_ab/$1.so -lrccl -pthread
rm -rf $OUT
echo $PKG/_ab/$1.so
