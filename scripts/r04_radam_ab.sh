# fused clip + RAdam: the round-3 kernel (variant library libsvae_oldradam.so) vs two vectors per thread with
# nontemporal moments: kernel probe alternating, the optimizer tests, then C2 / C4 benches alternating
cd "${GRAFT_REPO_ROOT:-/root/repo}"
OUT=gpurun_out/${1:-r04ra}; mkdir -p $OUT
OLD=SVAE_LIB=$PWD/sparse-vae_amd/sparse_vae/libsvae_oldradam.so
for v in A B A B; do
  if [ $v == A ]; then E=$OLD; else E=""; fi
  echo "== $v" >> $OUT/probe.log
  env $E timeout -k 10 200 python -u scripts/radam_probe.py >> $OUT/probe.log 2>&1 || exit $?
done
timeout -k 10 300 python -u -m pytest tests -m gpu -q -k "radam or clip or optim or step_matches" --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc == 0 ] || exit $rc
bash scripts/ab_bench.sh ${1:-r04ra} "$OLD" "SVAE_X=1" "c2 c4" 0 || exit $?
