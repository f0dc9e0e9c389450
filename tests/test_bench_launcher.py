"""`python bench.py --gpus N` starts N ranks itself (the reference reaches N GPUs through
Lightning's Trainer(gpus=N), train.py:63-64, 94): the spawn environment, failure propagation, the fail-fast
device-count check, and that the launcher process never initialises HIP. CPU only."""
import json
import os
import subprocess
import sys
import time

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402

_DUMP_ENV = ("import json, os, sys; "
             "keys = ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE', 'MASTER_ADDR', 'MASTER_PORT', "
             "'HSA_ENABLE_IPC_MODE_LEGACY'); "
             "open(os.path.join(sys.argv[1], 'rank%s.json' % os.environ['RANK']), 'w').write("
             "json.dumps({k: os.environ.get(k) for k in keys}))")


def test_spawned_ranks_get_the_torchrun_environment(tmp_path):
    rc = bench.launch_ranks(3, [sys.executable, '-c', _DUMP_ENV, str(tmp_path)])
    assert rc == 0
    envs = [json.loads((tmp_path / f'rank{r}.json').read_text()) for r in range(3)]
    for r, e in enumerate(envs):
        assert e['RANK'] == e['LOCAL_RANK'] == str(r)
        assert e['WORLD_SIZE'] == e['LOCAL_WORLD_SIZE'] == '3'
        assert e['MASTER_ADDR'] == '127.0.0.1'
        assert e['HSA_ENABLE_IPC_MODE_LEGACY'] == '0'
    assert len({e['MASTER_PORT'] for e in envs}) == 1 and int(envs[0]['MASTER_PORT']) > 0


def test_a_failing_rank_stops_the_others():
    # rank 1 fails at once; rank 0 would wait a minute (as in a collective whose partner died)
    child = [sys.executable, '-c', "import os, sys, time; r = int(os.environ['RANK']); "
                                   "sys.exit(7) if r == 1 else time.sleep(60)"]
    t0 = time.time()
    rc = bench.launch_ranks(2, child)
    assert rc == 7
    assert time.time() - t0 < 30


def test_too_few_gpus_fails_fast_without_touching_the_gpu():
    """On this GPU-less container (and on a 1-GPU box) `--gpus 2` must exit non-zero with the device-count
    message, and the launcher process must not have initialised HIP."""
    code = ("import runpy, sys, torch\n"
            "sys.argv = ['bench.py', '--gpus', '2', '--steps', '1', '--warmup', '0']\n"
            "try:\n"
            f"    runpy.run_path({os.path.join(ROOT, 'bench.py')!r}, run_name='__main__')\n"
            "except SystemExit as e:\n"
            "    print('HIP_INIT', torch.cuda.is_initialized(), flush=True)\n"
            "    raise\n")
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    r = subprocess.run([sys.executable, '-c', code], capture_output=True, text=True, env=env, timeout=600)
    if bench.device_count_in_child() >= 2:
        pytest.skip('this host has two GPUs')
    assert r.returncode != 0
    assert 'visible GPUs' in r.stderr
    assert 'HIP_INIT False' in r.stdout


def test_causal_useful_flops_count():
    # C2: dense 246.4 M per token; causal-useful subtracts 3 * nl * 2 * L * d
    dense = bench.flops_per_token(6, 512, 512)
    assert dense == pytest.approx(246.4e6, rel=1e-3)
    assert dense - bench.flops_per_token_causal(6, 512, 512) == 3 * 6 * 2 * 512 * 512
