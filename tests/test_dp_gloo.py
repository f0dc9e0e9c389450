"""Data-parallel gradient averaging over world_size 2 on CPU (gloo): the model's real bucketing code
(_dp_ready / _dp_finish over the gradient-ready flat arena), driven by the same ready() sequence the engine
backward emits. On the GPU the backend is 'nccl' (RCCL) and the engine calls ready() itself."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _ready_sequence(flat, hp):
    ends = [flat.end('output_layer.3.bias')]
    ends += [flat.end(f'z_projections.{i}.bias') for i in reversed(range(hp.num_layers))]
    ends.append(flat.end('q_of_z_given_x.linear.bias'))
    ends.append(flat.end('encoder.bottleneck.ffn_layer_norm.bias'))
    ends += [flat.end(f'encoder.middle_layers.{j}.ffn_layer_norm.bias') for j in reversed(range(hp.num_layers // 2 - 2))]
    ends.append(flat.end('encoder.first_layer.ffn_layer_norm.bias'))
    ends.append(flat.n_live)
    return ends


def _worker(rank, world, port, bucket_mb, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sparse-vae_amd'))
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    torch.manual_seed(100 + rank)                       # different init per rank: broadcast must unify
    hp = TransformerVAEHparams(d_model=128, num_layers=6, num_heads=8, sparse_self_attention=False)
    m = TransformerVAE(hp, device='cpu')
    m.enable_data_parallel(bucket_mb=bucket_mb)
    flat = m._flat
    g = torch.arange(flat.total, dtype=torch.float32) * 1e-6 + rank
    flat.grad.copy_(g / world)                         # the engine backward runs on loss / world
    for end in _ready_sequence(flat, m._ehp):
        m._dp_ready(end)
    m._dp_finish()
    live = flat.n_live
    q.put((rank, flat.master[:1000].numpy().copy(), flat.grad[:live].numpy().copy(), flat.grad[live:].numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize('world,bucket_mb', [(2, 0.5), (2, 64.0), (4, 0.5)])
def test_gradients_are_averaged_and_weights_broadcast(world, bucket_mb):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, bucket_mb, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranks = [[torch.from_numpy(a) for a in t] for _, *t in res]
    w0, g0, d0 = ranks[0]
    n = g0.numel()
    expect = torch.arange(n, dtype=torch.float32) * 1e-6 + (world - 1) / 2    # mean over ranks of (base + rank)
    torch.testing.assert_close(g0, expect, rtol=1e-6, atol=1e-6)
    for w1, g1, d1 in ranks[1:]:
        assert torch.equal(w0, w1)                     # rank 0's weights everywhere
        assert torch.equal(g0, g1)
        # gradients of parameters that never receive one (pos_linear) are not communicated
        assert not torch.equal(d0, d1)


GLOBAL_B = 8


def _sample_grad(total, s):
    """Per-sequence gradient of sample s of the global batch (distinct per sample and per element)."""
    return torch.arange(total, dtype=torch.float64) * 1e-6 * (s + 1) + torch.sin(torch.tensor(float(s))) * 3


def _worker_shard(rank, world, port, q):
    """The global batch of GLOBAL_B sequences sharded over `world` ranks (equal shards, RankBatchSampler's
    split): each rank's backward leaves its local mean / world in the arena, the model's buckets all-reduce."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sparse-vae_amd'))
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    hp = TransformerVAEHparams(d_model=128, num_layers=4, num_heads=8, sparse_self_attention=False)
    m = TransformerVAE(hp, device='cpu')
    m.enable_data_parallel(bucket_mb=0.25)
    flat = m._flat
    per = GLOBAL_B // world
    local = sum(_sample_grad(flat.total, s) for s in range(rank * per, (rank + 1) * per)) / per
    flat.grad.copy_((local / world).float())
    for end in _ready_sequence(flat, m._ehp):
        m._dp_ready(end)
    m._dp_finish()
    q.put((rank, flat.grad[:flat.n_live].numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [1, 2, 4, 8])
def test_world_sizes_give_the_global_batch_gradient(world):
    """ranks 1 / 2 / 4 / 8 over the same global batch give the same averaged gradient -- the
    global-batch mean -- on every rank."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_shard, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0 = torch.from_numpy(res[0][1]).double()
    n = g0.numel()
    expect = sum(_sample_grad(n, s) for s in range(GLOBAL_B)) / GLOBAL_B
    torch.testing.assert_close(g0, expect, rtol=2e-6, atol=2e-6)
    for _, g in res[1:]:
        assert torch.equal(torch.from_numpy(g), torch.from_numpy(res[0][1]))


class _FakeEngine:
    """Stands in for the HIP engine's backward on CPU: micro-step k on rank r adds g * G_k,r to the arena and
    emits the engine's ready() sequence when asked to."""

    def __init__(self, flat, ends, rank):
        self.flat, self.ends, self.rank, self.calls = flat, ends, rank, 0

    def backward(self, g, kl_weight, ready=None):
        self.calls += 1
        k = self.calls
        grad_k = torch.arange(self.flat.total, dtype=torch.float32) * 1e-6 * k + self.rank + 10 * k
        self.flat.grad.add_(g * grad_k)
        if ready is not None:
            for e in self.ends:
                ready(e)


def _worker_accum(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sparse-vae_amd'))
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    hp = TransformerVAEHparams(d_model=128, num_layers=4, num_heads=8, sparse_self_attention=False)
    m = TransformerVAE(hp, device='cpu')
    m.enable_data_parallel(bucket_mb=0.25)
    flat = m._flat
    m._engine = _FakeEngine(flat, _ready_sequence(flat, m._ehp), rank)
    m._kl_weight_used = 1.0
    # micro-step 1 (accumulation, no optimiser step after it) then micro-step 2 (optimiser step follows)
    for sync in (False, True):
        m.require_backward_grad_sync = sync
        m._run_backward(torch.tensor(1.0))
        if not sync:
            assert not m._dp['works'] and m._dp['start'] == 0     # nothing was communicated
    q.put((rank, flat.grad[:flat.n_live].numpy().copy()))
    dist.destroy_process_group()


@pytest.mark.parametrize('world', [2, 4])
def test_gradient_accumulation_reduces_once(world):
    """DP + accumulate_grad_batches=2 (the train.py default, train.py:16-23): the result is the rank-mean of
    each rank's summed micro-gradients -- the first micro-step's gradient is not reduced twice."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_accum, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    g0 = torch.from_numpy(res[0][1])
    n = g0.numel()
    ar = torch.arange(n, dtype=torch.float32) * 1e-6
    # sum over k = 1, 2 of (ar * k + rank + 10 k), averaged over the ranks
    expect = ar * 3 + (world - 1) / 2 * 2 + 30
    torch.testing.assert_close(g0, expect, rtol=1e-6, atol=1e-5)
    for _, g in res[1:]:
        assert torch.equal(g0, torch.from_numpy(g))


def _fake_sumsq(g, n, part):
    part.zero_()
    part[0] = g[:n].double().pow(2).sum().float()


def _fake_clip(g, n, part, max_norm, norm_out=None):
    norm = part.double().sum().sqrt().item()
    g[:n].mul_(min(1.0, max_norm / (norm + 1e-6)))


def _worker_clip(rank, world, port, q):
    """An accumulation micro-step under DP: the arena holds G_local / world (the backward ran on loss / world);
    on_after_backward must clip the unscaled G_local at the threshold (DDP's no_sync micro-step) and log its
    norm. The device kernels (sumsq / clip_grad) are replaced by torch equivalents on CPU; the host logic --
    which threshold, which norm is logged -- is the model's own."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'sparse-vae_amd'))
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    from sparse_vae import kernels as K
    K.sumsq, K.clip_grad = _fake_sumsq, _fake_clip
    hp = TransformerVAEHparams(d_model=128, num_layers=4, num_heads=8, sparse_self_attention=False,
                               grad_clip_threshold=5.0)
    m = TransformerVAE(hp, device='cpu')
    m.enable_data_parallel(bucket_mb=0.25)
    flat = m._flat
    n = flat.n_live
    v = torch.ones(n) * (rank + 1)
    v *= 20.0 * (rank + 1) / v.norm()                    # |G_local| = 20 (rank 0), 40 (rank 1): both above 5
    flat.grad[:n].copy_(v / world)
    m.require_backward_grad_sync = False
    m.on_after_backward()
    logged_norm = float(m.logged['grad_norm'])
    clipped = flat.grad[:n].clone()
    # the sync micro-step's norm is of the all-reduced (rank-mean) arena: no rescale
    m.require_backward_grad_sync = True
    flat.grad[:n].copy_(v)
    m.on_after_backward()
    sync_norm = float(m.logged['grad_norm'])
    # logged scalars: rank means
    m.logged.update({'train_nll': torch.tensor(1.0 + rank), 'train_kl': torch.tensor(10.0 * (rank + 1)),
                     'loss': torch.tensor(3.0 - rank)})
    m.reduce_logged()
    vals = m.logged_values()
    red = {k: vals[k] for k in ('train_nll', 'train_kl', 'loss')}
    q.put((rank, logged_norm, (clipped.double() * world).norm().item(), (clipped.double() * world / v.double()).std().item(), sync_norm, red))
    dist.destroy_process_group()


def test_micro_step_clip_uses_the_unscaled_local_gradient():
    """with world 2 and accumulate_grad_batches > 1 the non-sync micro-step's clip must compare the
    local gradient G (not G / world) with grad_clip_threshold, and log |G|; the logged loss / nll / kl are
    averaged over the ranks once per optimiser step."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_clip, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=240) for _ in range(world)], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, logged_norm, clipped_local_norm, ratio_std, sync_norm, red in res:
        assert logged_norm == pytest.approx(20.0 * (rank + 1), rel=1e-5)
        assert clipped_local_norm == pytest.approx(5.0, rel=1e-5)      # G clipped to the threshold, not 5 * world
        assert ratio_std < 1e-6                                          # a uniform scale
        assert sync_norm == pytest.approx(20.0 * (rank + 1), rel=1e-5)
        assert red == pytest.approx({'train_nll': 1.5, 'train_kl': 15.0, 'loss': 2.5})
