export TMPDIR=/tmp; mkdir -p gpurun_out/gp2
for g in 0 4 8 16; do SVAE_GEMM_GROUP=$g timeout -k 10 120 python3 scripts/gemm_probe.py all >> gpurun_out/gp2/probe.log 2>&1 || exit 1; done
SVAE_GEMM_GROUP=8 timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex gemm256 -f csv -d gpurun_out/gp2/fetch -o run -- python3 scripts/gemm_probe.py > gpurun_out/gp2/f.log 2>&1
grep -v amdgpu.ids gpurun_out/gp2/probe.log
