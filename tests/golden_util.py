"""Helpers shared by the tests: load a golden fixture and rebuild its inputs/weights."""
import os

import numpy as np
import torch

from oracle.params import HParams, init_params

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')
CONFIG_NAMES = ['tiny', 'tiny_pad', 'small6_pad', 'hd96', 'c2shape', 'c4shape', 'c5shape']


def load(name):
    with np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def setup(name):
    g = load(name)
    d, H, NL, L, B, padded, seed = [int(v) for v in g['cfg']]
    hp = HParams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64, kl_weight=float(g['kl_weight']))
    params = init_params(hp, seed)
    ids = torch.from_numpy(g['ids'].astype(np.int64))
    return g, hp, params, ids


GEN_NAMES = ['gen_dense', 'gen_dense_nopen', 'gen_sparse']


def setup_gen(name):
    """A generation fixture (make_golden.generation_vectors): hparams, weights (tied embedding scaled by
    emb_scale for peaked logits) and the latent z [B, 1, 64]."""
    g = load(name)
    d, H, NL, window, B, T, seed = [int(v) for v in g['cfg']]
    hp = HParams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64, kl_weight=1.0, attn_window=window)
    params = init_params(hp, seed)
    params['input_layer.0.weight'] = params['input_layer.0.weight'] * float(g['emb_scale'])
    return g, hp, params, torch.from_numpy(g['z'])


def setup_iw():
    g = load('iw')
    d, H, NL, L, B, seed = [int(v) for v in g['cfg']]
    hp = HParams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64, kl_weight=1.0)
    params = init_params(hp, seed)
    ids = torch.from_numpy(g['ids'].astype(np.int64))
    return g, hp, params, ids


def ce_logits(a, u, w, s):
    """The chunked-CE fixture's logits (make_golden.ce_vectors): a (x) w + u (x) s, [B, L-1, V] f32."""
    logits = a[:, :, None] * w[None, None, :]
    logits.addcmul_(u[:, :, None], s[None, None, :])
    return logits


def setup_ce():
    g = load('ce_chunked')
    t = {k: torch.from_numpy(g[k]) for k in ('a', 'u', 'w', 's', 'tok_w')}
    return g, t, torch.from_numpy(g['labels'].astype(np.int64))
