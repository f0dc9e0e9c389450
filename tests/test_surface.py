"""The reference-compatible Python surface (CPU): module tree / state_dict keys, hparams, presets, CLI
parsing, the synthetic data module's wire format, the flat parameter layout invariants the kernels rely on,
and the optimiser's host arithmetic."""
import dataclasses
import json
import os
import sys

import numpy as np
import pytest
import torch

from golden_util import GOLDEN

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize('name,d,H,nl', [('tiny', 128, 8, 4), ('small6_pad', 256, 4, 6), ('hd96', 384, 4, 6),
                                         ('c2shape', 512, 8, 6)])
def test_state_dict_matches_reference(name, d, H, nl):
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    ref = json.load(open(os.path.join(GOLDEN, 'reference_keys.json')))[name]
    m = TransformerVAE(TransformerVAEHparams(d_model=d, num_layers=nl, num_heads=H, sparse_self_attention=False),
                       device='cpu')
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    assert {k: list(v.shape) for k, v in sd.items()} == ref
    # tied weights share storage (transformer_language_model.py:62-63, transformer_vae.py:30-31)
    assert sd['output_layer.3.weight'].data_ptr() == sd['input_layer.0.weight'].data_ptr()
    assert sd['encoder_input_layer.0.weight'].data_ptr() == sd['input_layer.0.weight'].data_ptr()


def test_load_state_dict_roundtrip_and_views():
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    hp = TransformerVAEHparams(d_model=128, num_layers=4, num_heads=8, sparse_self_attention=False)
    a = TransformerVAE(hp, device='cpu')
    b = TransformerVAE(hp, device='cpu')
    b.load_state_dict(a.state_dict())
    for (n1, p1), (n2, p2) in zip(a.state_dict().items(), b.state_dict().items()):
        assert torch.equal(p1, p2)
    # every parameter is a view into the flat arena
    base = b._flat.master.data_ptr()
    end = base + b._flat.master.numel() * 4
    for p in b.parameters():
        assert base <= p.data_ptr() < end


def test_hparams_fields_match_reference_names():
    from sparse_vae import TransformerVAEHparams
    names = {f.name for f in dataclasses.fields(TransformerVAEHparams)}
    for n in ['d_model', 'num_heads', 'num_layers', 'latent_depth', 'sparse_self_attention', 'attn_window_size',
              'grad_checkpointing', 'tie_embedding_weights', 'init_scale', 'lr', 'grad_clip_threshold',
              'kl_weight', 'kl_weight_start', 'kl_weight_end', 'kl_annealing_steps', 'lr_decay_steps',
              'base_batch_size', 'early_stopping_metric', 'input_dropout', 'd_embedding', 'cross_attention']:
        assert n in names, n
    hp = TransformerVAEHparams()
    assert hp.sparse_self_attention is True and hp.d_model == 512 and hp.num_layers == 6   # reference defaults


def test_perceiver_needs_four_layers():
    from sparse_vae import TransformerVAE, TransformerVAEHparams
    with pytest.raises(AssertionError):
        TransformerVAE(TransformerVAEHparams(d_model=128, num_layers=2, num_heads=8, sparse_self_attention=False),
                       device='cpu')


def test_flat_layout_invariants():
    """q/k/v weights and biases adjacent (one fused GEMM operand), LayerNorm weight|bias adjacent, gradient-ready
    order, pos_linear (never receives a gradient) after the live prefix."""
    from oracle.params import HParams
    from sparse_vae.engine import FlatParams
    hp = HParams(d_model=256, num_heads=4, num_layers=6)
    f = FlatParams(hp, 'cpu')
    d = 256
    for pre in ['decoder_layers.0.attention.', 'encoder.middle_layers.0.attention.',
                'encoder.middle_layers.0.cross_attention.']:
        q = f.offsets[pre + 'q_linear.weight'][0]
        assert f.offsets[pre + 'k_linear.weight'][0] == q + d * d
        assert f.offsets[pre + 'v_linear.weight'][0] == q + 2 * d * d
        qb = f.offsets[pre + 'q_linear.bias'][0]
        assert f.offsets[pre + 'k_linear.bias'][0] == qb + d and f.offsets[pre + 'v_linear.bias'][0] == qb + 2 * d
    for ln in ['decoder_layers.3.attn_layer_norm', 'encoder.first_layer.ffn_layer_norm', 'output_layer.2']:
        assert f.offsets[ln + '.bias'][0] == f.offsets[ln + '.weight'][0] + d
    order = [f.offsets[n][0] for n in ['output_layer.0.weight', 'decoder_layers.5.ffn.0.weight',
                                       'decoder_layers.0.ffn.0.weight', 'q_of_z_given_x.linear.weight',
                                       'encoder.bottleneck.ffn.0.weight', 'encoder.first_layer.ffn.0.weight',
                                       'input_layer.0.weight']]
    assert order == sorted(order)
    assert all(f.offsets[n][0] >= f.n_live for n in f.offsets if 'pos_linear' in n)
    assert all(f.offsets[n][0] < f.n_live for n in f.live_names)
    assert all(off % 64 == 0 for off, _ in f.offsets.values())


def test_context_layernorm_layout_follows_the_batching_switch(monkeypatch):
    """With >= 2 encoder middle layers the context LayerNorms (one per middle layer, all over x_emb) are batched: their
    [weight | bias] pairs sit together after every middle layer (their gradients complete in one backward pass after the
    middle layers) and before the first layer; SVAE_CTX_LN_BATCH=0 keeps each inside its layer."""
    from oracle.params import HParams
    from sparse_vae.engine import FlatParams
    hp = HParams(d_model=256, num_heads=4, num_layers=12)   # 6 encoder layers: 4 middle
    f = FlatParams(hp, 'cpu')
    assert f.ctx_batched
    ctx = [f.offsets[f'encoder.middle_layers.{j}.context_layer_norm.weight'][0] for j in range(4)]
    mids = [f.offsets[f'encoder.middle_layers.{j}.ffn_layer_norm.bias'][0] for j in range(4)]
    first = f.offsets['encoder.first_layer.attention.k_linear.weight'][0]
    assert min(ctx) > max(mids) and max(ctx) < first
    for j in range(4):
        n = f'encoder.middle_layers.{j}.context_layer_norm'
        assert f.offsets[n + '.bias'][0] == f.offsets[n + '.weight'][0] + 256
    monkeypatch.setenv('SVAE_CTX_LN_BATCH', '0')
    g = FlatParams(hp, 'cpu')
    assert not g.ctx_batched
    for j in range(4):
        pre = f'encoder.middle_layers.{j}.'
        assert g.offsets[pre + 'cross_attn_layer_norm.bias'][0] < g.offsets[pre + 'context_layer_norm.weight'][0] \
            < g.offsets[pre + 'ffn.0.weight'][0]
    assert set(f.offsets) == set(g.offsets)


def test_presets_and_cli_parsing():
    sys.path.insert(0, ROOT)
    import train
    from hparam_presets import hparam_presets
    for name in ['tiny', 'c2', 'c4', 'c5', 'dense-benchmark', 'sparse-benchmark', 'wikipedia', 'pg19']:
        assert name in hparam_presets
    cfg = train.build_config(['model.d_model=256', 'model.lr=1e-3', 'data.seq_len=64', 'preset=tiny'])
    # the preset is merged AFTER the dotlist and wins (train.py:57-61 in the reference)
    assert cfg['model']['d_model'] == 128 and cfg['model']['lr'] == 3e-4 and cfg['data']['seq_len'] == 128
    cfg = train.build_config(['model.kl_weight=0.5', 'trainer.max_steps=3'])
    assert cfg['model']['kl_weight'] == 0.5 and cfg['trainer']['max_steps'] == 3
    assert cfg['trainer']['accumulate_grad_batches'] == 2        # train.py:16-23 default


def test_synthetic_batch_wire_format():
    from sparse_vae import TextDataModule, PaddedTensor
    dm = TextDataModule(dataset_name='synthetic', seq_len=512, batch_size=4, padded=True)
    b = dm.synthetic_batch(3)
    ids = b['token_ids']
    assert isinstance(ids, PaddedTensor) and ids.dtype == torch.int16 and ids.shape == (4, 512)
    raw = ids.as_raw()
    assert (raw[:, 0] == 1).all()
    for i, n in enumerate(b['num_tokens'].tolist()):
        assert raw[i, n - 1] == 2 and (raw[i, n:] == 0).all() and (raw[i, :n] != 0).all()
    assert torch.equal(ids.padding, raw.eq(0))
    assert torch.equal(b['num_bytes'], b['num_tokens'])
    # same index -> same batch (deterministic)
    assert torch.equal(dm.synthetic_batch(3)['token_ids'].as_raw(), raw)


def test_pad_pack_rounds_to_multiple_of_512():
    from sparse_vae import TextDataModule
    dm = TextDataModule(dataset_name='synthetic')
    out = dm.pad_pack([torch.arange(1, 600, dtype=torch.int16), torch.arange(1, 10, dtype=torch.int16)])
    assert out.shape == (2, 1024) and out[1, 9:].eq(0).all() and out[0, 598] == 599
    coll = dm.collate([{'text': np.arange(1, 20), 'num_tokens': 19, 'num_bytes': 40}])
    assert coll['token_ids'].shape == (1, 512) and coll['token_ids'].dtype == torch.int16


def test_radam_host_scalars_follow_reference():
    """The per-step scalars the fused kernel receives reproduce rectified_adam.py:26-37 / :82."""
    import oracle
    from sparse_vae.core.rectified_adam import RAdam
    group = {'lr': 3e-3, 'betas': (0.9, 0.999), 'eps': 1e-6, 'weight_decay': 0.01}
    opt = RAdam.__new__(RAdam)
    opt.max_grad_norm = 150.0
    g = torch.from_numpy(np.linspace(-1, 1, 50).astype(np.float32))
    p = torch.from_numpy(np.linspace(2, -3, 50).astype(np.float32))
    m, v = torch.zeros(50), torch.zeros(50)
    st = oracle.RAdamState()
    ref = {'p': p.clone()}
    for s in range(7):
        lr, bcm, bcv, rho_ok, b1, b2, eps, wd, mx = opt.step_scalars(group)
        group['step'] += 1
        # the kernel's arithmetic, restated on the host
        m = m * b1 + (1 - b1) * g
        v = v * b2 + (1 - b2) * g * g
        p = p * (1 - lr * wd)
        p = p - (lr / bcm) * (m / (v.sqrt() / bcv + eps) if rho_ok else m)
        ref = oracle.radam_step(ref, {'p': g}, st, lr=3e-3, weight_decay=0.01)
        np.testing.assert_allclose(p.numpy(), ref['p'].numpy(), rtol=1e-6, atol=1e-7)


def test_cosine_decay_and_kl_anneal():
    from sparse_vae.core import cosine_decay
    import oracle
    for s in (0, 10, 500, 999):
        assert cosine_decay(1000, s) == oracle.cosine_decay(1000, s)
    with pytest.raises(KeyboardInterrupt):
        cosine_decay(1000, 1000)
    from sparse_vae.core.continuous_autoencoder import ContinuousVAEHooks
    from sparse_vae.core.language_model import AttributeDict

    class M(ContinuousVAEHooks):
        hparams = AttributeDict(kl_weight=0.3, kl_weight_start=0.3, kl_weight_end=1.0, kl_annealing_steps=100)
        global_step = 40

    mm = M()
    mm.anneal_kl()
    assert abs(mm.hparams.kl_weight - oracle.kl_anneal(0.3, 0.3, 1.0, 100, 40)) < 1e-12
