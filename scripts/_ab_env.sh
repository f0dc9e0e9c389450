# A/B of an environment switch in ONE box session: bench.py with each "VAR=value" setting, twice each, alternating
#   bash scripts/_ab_env.sh "SVAE_HEAD_DW_KC=1" "SVAE_HEAD_DW_KC=0"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for rep in 1 2; do
  for setting in "$@"; do
    echo "== $setting"
    env $setting timeout -k 10 200 python3 -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-parity 2>&1 | tail -1 | cut -c1-200 || exit 1
  done
done
