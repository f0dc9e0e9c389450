cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/r04o
SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_kw1.so timeout -k 10 300 python -u scripts/kw_diag2.py > gpurun_out/r04o/kw_diag2.log 2>&1
