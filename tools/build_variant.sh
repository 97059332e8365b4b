#!/bin/bash
# Build the engine with extra compiler flags into mm-vae_amd/lib_NAME/libmmvae.so (A/B with
# MMVAE_LIB=mm-vae_amd/lib_NAME/libmmvae.so).   Usage: bash tools/build_variant.sh NAME "FLAGS"
NAME=$1; FLAGS=$2
cd "$(dirname "$0")/../mm-vae_amd"
mkdir -p build_$NAME lib_$NAME
for f in $(sed -n "s/^SRCS *:= *//p" Makefile | tr " " "\n" | sed -n "s|csrc/\(.*\)\.hip|\1|p"); do
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -fPIC -munsafe-fp-atomics -I/opt/rocm/include $FLAGS \
    -c csrc/$f.hip -o build_$NAME/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 build_$NAME/*.o -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o lib_$NAME/libmmvae.so
ls -la lib_$NAME/libmmvae.so
