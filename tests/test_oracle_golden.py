"""Pin the CPU oracle (oracle/) against golden vectors produced by the real reference
(tests/golden/make_golden.py). CPU only."""
import json
import os

import numpy as np
import pytest
import torch

import oracle
from oracle.params import param_shapes, TIED_ALIASES
from golden_util import GOLDEN, CONFIG_NAMES, load, setup


def _rel(a, b):
    return abs(float(a) - float(b)) / max(abs(float(b)), 1e-30)


@pytest.mark.parametrize('name', CONFIG_NAMES)
def test_param_inventory_matches_reference(name):
    with open(os.path.join(GOLDEN, 'reference_keys.json')) as f:
        ref = json.load(f)[name]
    g, hp, params, _ = setup(name)
    mine = {k: list(v) for k, v in param_shapes(hp).items()}
    for alias in TIED_ALIASES:
        mine[alias] = mine['input_layer.0.weight']
    assert mine == ref


@pytest.mark.parametrize('name', CONFIG_NAMES)
def test_training_step_matches_reference(name):
    torch.set_num_threads(min(8, os.cpu_count()))
    g, hp, params, ids = setup(name)
    p = {k: v.clone().requires_grad_(True) for k, v in params.items()}
    out = oracle.training_step(p, hp, ids, torch.from_numpy(g['lens']), torch.from_numpy(g['eps']),
                               eps_marginal=torch.from_numpy(g['eps10']))
    out['loss'].backward()
    assert _rel(out['loss'].item(), g['loss']) < 1e-6
    assert _rel(out['nll'].item(), g['train_nll']) < 1e-6
    assert _rel(out['train_kl'].item(), g['train_kl']) < 1e-5
    assert abs(out['mutual_info'].item() - g['mutual_info']) < 1e-4 * max(1.0, abs(g['mutual_info']))
    np.testing.assert_allclose(out['mu'].detach().numpy().reshape(g['mu'].shape), g['mu'], rtol=1e-5, atol=1e-6)
    names = [str(n) for n in g['grad_names']]
    have = {k for k, v in p.items() if v.grad is not None}
    assert set(names) == have            # pos_linear etc. receive no gradient in either
    for n in names:
        gr = p[n].grad.detach().flatten().double().numpy()
        assert _rel(np.linalg.norm(gr), g['gnorm/' + n]) < 1e-4, n
        np.testing.assert_allclose(gr[g['gidx/' + n]], g['gval/' + n], rtol=2e-3, atol=2e-7 + 2e-4 * np.abs(g['gval/' + n]).max())


@pytest.mark.parametrize('name', ['tiny', 'small6_pad'])
def test_argmax_reconstruction_matches_reference(name):
    g, hp, params, ids = setup(name)
    with torch.no_grad():
        pad = ids.eq(0)
        x = torch.nn.functional.embedding(ids, params['input_layer.0.weight'])
        mu = torch.from_numpy(g['mu']).reshape(-1, 1, 64)
        logits = oracle.reconstruct(params, x, mu, pad, hp)[..., :-1, :]
    am = logits.argmax(-1).numpy()
    assert (am == g['argmax']).all()
    np.testing.assert_allclose(logits[0, [0, ids.shape[1] // 2]].numpy(), g['logit_rows'], rtol=1e-4, atol=1e-5)


def test_rotary_matches_reference():
    g = load('ops')
    for i in range(3):
        start, max_pos = [int(v) for v in g[f'rot{i}_meta']]
        out = oracle.rotary(torch.from_numpy(g[f'rot{i}_in']), start, max_pos)
        np.testing.assert_array_equal(out.numpy(), g[f'rot{i}_out'])


def test_radam_matches_reference():
    g = load('ops')
    params = {'p0': torch.from_numpy(g['radam_p0']), 'p1': torch.from_numpy(g['radam_p1'])}
    st = oracle.RAdamState()
    for s in range(8):
        grads = {'p0': torch.from_numpy(g[f'radam_g0_{s}']), 'p1': torch.from_numpy(g[f'radam_g1_{s}'])}
        params = oracle.radam_step(params, grads, st, lr=3e-3, weight_decay=0.01)
        np.testing.assert_allclose(params['p0'].numpy(), g[f'radam_out0_{s}'], rtol=1e-6, atol=1e-7)
        np.testing.assert_allclose(params['p1'].numpy(), g[f'radam_out1_{s}'], rtol=1e-6, atol=1e-7)


def test_cosine_decay_matches_reference():
    g = load('ops')
    got = [oracle.cosine_decay(1000, s) for s in (0, 1, 250, 500, 999)]
    np.testing.assert_allclose(got, g['cosine'], rtol=0, atol=0)
    with pytest.raises(KeyboardInterrupt):
        oracle.cosine_decay(1000, 1000)


def test_sparse_layout_matches_reference():
    """oracle.sparse_layout == SparseAttention.get_master_layout (sparse_attention.py:39-60) of the reference,
    and Attention(sparse=w) builds SparseAttention(window_size=w, block_size=32, causal, include_cls)."""
    g = load('sparse')
    for w in (1, 2, 3, 4, 6):
        ref = g[f'layout_w{w}']
        nb = ref.shape[-1]
        ours = oracle.sparse_layout(nb, w).to(torch.int8).numpy()
        for h in range(ref.shape[0]):
            np.testing.assert_array_equal(ours, ref[h])
    for w in (4, 2):
        np.testing.assert_array_equal(g[f'window_of_sparse_{w}'], [w, 32, 1, 1])
    # the mask the kernels implement: key k <= q visible iff k < 32 or k // 32 >= q // 32 - (w - 1)
    L, w = 320, 3
    m = oracle.sparse_mask(L, w)
    q, k = torch.meshgrid(torch.arange(L), torch.arange(L), indexing='ij')
    vis = (k <= q) & ((k < 32) | (k // 32 >= q // 32 - (w - 1)))
    assert torch.equal(~m, vis)


def test_sparse_rotary_table_matches_reference():
    """The engine's host-built rotary table at SparseAttention's base 2 * 4 * 32 = 256 reproduces the reference's
    encode_position_rotary(max_pos=256) (golden rot2: positions 0..299, d 32)."""
    from sparse_vae.engine import rotary_table
    g = load('ops')
    start, max_pos = [int(v) for v in g['rot2_meta']]
    assert (start, max_pos) == (0, 256)
    x = torch.from_numpy(g['rot2_in'])[0]
    tab = rotary_table(x.shape[0], x.shape[1], max_pos)
    c, s = tab[..., 0], tab[..., 1]
    a, b = x[:, 0::2], x[:, 1::2]
    out = torch.stack([a * c + (-b) * s, b * c + a * s], -1).flatten(-2)
    np.testing.assert_allclose(out.numpy(), g['rot2_out'][0], rtol=0, atol=2e-6)


def test_robust_cross_entropy_chunked_branch_pinned():
    """The > 2^30-element branch (language_model.py:163-170): 2 sequence chunks, mean of per-chunk means, and the
    class-weighted form (val_bpb), against the reference's own values on the same 4.3 GB of logits."""
    from golden_util import ce_logits, setup_ce
    torch.set_num_threads(min(8, os.cpu_count()))
    g, t, labels = setup_ce()
    logits = ce_logits(t['a'], t['u'], t['w'], t['s'])
    assert -(-logits.numel() // 2 ** 30) == 2
    with torch.no_grad():
        nll = oracle.robust_cross_entropy(logits, labels).item()
        wnll = oracle.robust_cross_entropy(logits, labels, weight=t['tok_w']).item()
    del logits
    assert abs(nll - float(g['nll'])) <= 1e-6 * abs(float(g['nll']))
    assert abs(wnll - float(g['wnll'])) <= 1e-6 * abs(float(g['wnll']))
    assert abs(float(g['nll']) - float(g['single_mean'])) > 1e-3   # the chunking matters at this bar
