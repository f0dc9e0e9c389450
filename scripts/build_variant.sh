#!/bin/bash
# Build an A/B variant of libsvae: recompile ONE source with extra flags, link with the in-tree objects of the rest.
#   bash scripts/build_variant.sh NAME SOURCE.hip [extra hipcc flags...]  ->  sparse_vae/libsvae_NAME.so
set -e
cd "$(dirname "$0")/../sparse-vae_amd"
name=$1; src=$2; shift 2
make -s
base=$(basename "$src" .hip)
mkdir -p build/var
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics -Wall -Wno-unused-function \
  -fno-honor-nans "$@" -c "csrc/$base.hip" -o "build/var/${base}_$name.o"
objs=$(ls build/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o "sparse_vae/libsvae_$name.so" $objs "build/var/${base}_$name.o"
echo "built sparse_vae/libsvae_$name.so"
