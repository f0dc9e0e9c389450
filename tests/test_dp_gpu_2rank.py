"""Two data-parallel ranks of the real GPU training step (tests/dp_two_rank_worker.py, one process per rank, both on
the box's single GPU, gloo backend): the engine backward's ready() callbacks launch the model's bucketed async
all-reduces (1 MB buckets, so many are in flight) and the backward runs on loss / world, so the all-reduced gradient
must equal the single-process gradient of the whole batch (each rank holds half the sequences; the reference's loss
is a mean over equal-length sequences, so the mean over ranks of the half-batch losses is the full-batch loss).
This is the N > 1 path of bench.py / Trainer.fit with gloo standing in for RCCL (one rank per GPU); the 2..8-GPU RCCL
runs are the driver's."""
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_data_parallel_step_matches_full_batch(tmp_path):
    world, port = 2, _port()
    outs = [str(tmp_path / f'rank{r}.pt') for r in range(world)]
    env = dict(os.environ, MASTER_ADDR='127.0.0.1')
    # child processes (never an exec of this GPU-initialised process); each bounded in time
    procs = [subprocess.Popen([sys.executable, os.path.join(HERE, 'dp_two_rank_worker.py'), str(r), str(world),
                               str(port), outs[r]], env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT)
             for r in range(world)]
    logs = []
    for p in procs:
        try:
            logs.append(p.communicate(timeout=150)[0].decode(errors='replace'))
        except subprocess.TimeoutExpired:
            for q in procs:
                q.kill()
            raise
    for p, log in zip(procs, logs):
        assert p.returncode == 0, log[-3000:]
    r0, r1 = (torch.load(o, weights_only=True) for o in outs)
    assert torch.equal(r0['w'], r1['w'])                         # rank 0's weights were broadcast
    assert torch.equal(r0['grad'], r1['grad'])                   # every rank holds the same averaged gradient
    mean_loss = 0.5 * (r0['loss'] + r1['loss'])
    assert abs(mean_loss - r0['ref_loss']) / abs(r0['ref_loss']) < 1e-5
    g, ref = r0['grad'].double(), r0['ref_grad'].double()
    # (split-K slicing of the weight gradients differs between the half and the full batch, so the sums are not
    # bitwise equal; a DP bug -- a missing 1/world, a bucket reduced twice or skipped -- is an O(1) error)
    assert ((g - ref).norm() / ref.norm()).item() < 1e-4
    cos = (g @ ref / (g.norm() * ref.norm())).item()
    assert cos > 0.99999
    # two accumulated micro-steps per rank (no_sync on the first): the rank mean of the summed micro-gradients
    assert torch.equal(r0['acc_grad'], r1['acc_grad'])
    g, ref = r0['acc_grad'].double(), r0['ref_acc_grad'].double()
    assert ((g - ref).norm() / ref.norm()).item() < 1e-4
    assert (g @ ref / (g.norm() * ref.norm())).item() > 0.99999
