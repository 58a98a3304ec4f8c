#!/bin/bash
# Build an experimental libm3s variant: build_variant.sh NAME "-DMACRO=..."  ->  lightweight-mast3r-slam_amd/lib/exp/libm3s_NAME.so
# (load it with M3S_LIB=...; the shipped library is always csrc/Makefile's ../lib/libm3s.so)
set -e
cd "$(dirname "$0")/../lightweight-mast3r-slam_amd/csrc"
make -s -j8 >/dev/null
mkdir -p ../lib/exp build/exp
HIPCC=/opt/rocm/bin/hipcc
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -ffp-contract=off -fno-slp-vectorize $2 -c refine.hip -o build/exp/refine_$1.o
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -ffp-contract=off -fno-slp-vectorize $2 -c track.hip -o build/exp/track_$1.o
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -munsafe-fp-atomics -ffp-contract=off $2 -c ba.hip -o build/exp/ba_$1.o
$HIPCC --offload-arch=gfx950 -O3 -fPIC -std=c++17 -ffp-contract=off $2 -c retrieval.hip -o build/exp/retrieval_$1.o
$HIPCC --offload-arch=gfx950 -shared -fPIC -o ../lib/exp/libm3s_$1.so build/matching.o build/exp/refine_$1.o build/exp/track_$1.o build/exp/ba_$1.o build/ba_dense.o build/peaks.o build/exp/retrieval_$1.o build/ba_pattern.o build/abi.o
echo built ../lib/exp/libm3s_$1.so
