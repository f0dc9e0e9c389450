# same box: the late round-4 launch-level changes off (LayerNorm forward one row per wave, one slab reduction per
# GEMM) vs the defaults, alternating, three pairs
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04v}; mkdir -p $OUT
A="SVAE_LN_FWD_BLOCKS=0 SVAE_SLAB2=0"
for i in 1 2 3; do
  for v in A B; do
    if [ $v == A ]; then E=$A; else E=""; fi
    env $E timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-parity > $OUT/bench_${v}_$i.log 2>&1 || exit $?
    echo "c2 $v ($E): $(tail -1 $OUT/bench_${v}_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])') ms/step"
  done
done
