"""The N-rank bench path end to end on the GPU box: `bench.py --gpus 2` launches two ranks itself;
on a 1-GPU box they share the GPU (SVAE_BENCH_SHARE_GPUS=1) over gloo, so the launcher, the rank environment, the
data-parallel step, the max-over-ranks timing and the same-run scaling figure all run on hardware. The line is
labelled a rehearsal; the RCCL run is the driver's multi-GPU bench."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_two_rank_bench_rehearsal():
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'MASTER_PORT')}
    env.update(SVAE_BENCH_SHARE_GPUS='1', SVAE_DIST_BACKEND='gloo')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2', '--steps', '2', '--warmup', '1',
                        '--config', 'tiny'], capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, r.stdout          # rank 0 prints exactly one line
    res = json.loads(lines[0])
    assert res['n_gpus'] == 2 and res['config']['parallelism'] == 'dp2' and res['config']['global_batch'] == 128
    assert res['value'] > 0 and 'rehearsal' in res
    assert 0 < res['scaling_efficiency']['value'] < 10
    # the all-reduce tail the backward did not hide (HIP events on the compute stream, max over ranks)
    assert res['exposed_comm_ms']['value'] >= 0 and 0 <= res['exposed_comm_ms']['fraction_of_step'] < 10
    assert 'cpu_baseline' not in res and 'parity' not in res
