export TMPDIR=/tmp; mkdir -p gpurun_out/gp4
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -k gemm > gpurun_out/gp4/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/gp4/pytest.log; [ $rc = 0 ] || exit $rc
for cfg in "SVAE_GEMM_PERSIST=0" "SVAE_GEMM_DESYNC=0 SVAE_GEMM_RELAX=0" "SVAE_GEMM_RELAX=0" "SVAE_GEMM_DESYNC=0" "SVAE_GEMM_X=1" "SVAE_GEMM_DESYNC=1" "SVAE_GEMM_DESYNC=4"; do
  echo "== $cfg" >> gpurun_out/gp4/probe.log
  env $cfg timeout -k 10 120 python3 scripts/gemm_probe.py all 2>&1 | grep -v amdgpu.ids >> gpurun_out/gp4/probe.log || exit 1
done
cat gpurun_out/gp4/probe.log
