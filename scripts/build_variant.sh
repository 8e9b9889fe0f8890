#!/bin/bash
# build an experimental libgossip_hip.so variant: build_variant.sh NAME "-DFLAG=..."
# output: gossip-protocol-with-power-law_amd/_ab/NAME.so (git-ignored, travels to the GPU box)
set -e
cd "$(dirname "$0")/.."
PKG=gossip-protocol-with-power-law_amd
OUT=$PKG/_ab/$1
mkdir -p $OUT
F="-O3 -std=c++17 -fPIC -Wall -Wno-unused-result --offload-arch=gfx950 $2"
/opt/rocm/bin/hipcc $F -c $PKG/csrc/gossip_engine.hip -o $OUT/ge.o &
/opt/rocm/bin/hipcc $F -c $PKG/csrc/graph_build.hip -o $OUT/gb.o &
/opt/rocm/bin/hipcc $F -c $PKG/csrc/checkpoint.hip -o $OUT/ck.o &
/opt/rocm/bin/hipcc $F -c $PKG/csrc/partition.hip -o $OUT/pt.o &
/opt/rocm/bin/hipcc $F -c $PKG/csrc/bitcount.hip -o $OUT/bc.o &
wait
/opt/rocm/bin/hipcc $F -shared $OUT/ge.o $OUT/gb.o $OUT/ck.o $OUT/pt.o $OUT/bc.o -o $PKG/_ab/$1.so -lrccl -pthread
rm -rf $OUT
echo $PKG/_ab/$1.so
