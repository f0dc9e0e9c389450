#!/bin/bash
# A/B of libsvae builds (SVAE_LIB) under a kernel trace of the C2 bench; args: variant names (libsvae_<v>.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in "$@"; do
  SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats -f csv \
    -d gpurun_out/ab_$v -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-parity \
    > gpurun_out/ab_$v.log 2>&1 || exit 1
done
