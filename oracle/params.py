"""ORACLE — test infrastructure only (see oracle/__init__.py).

Parameter inventory of the reference TransformerVAE and a portable, counter-based weight
generator so that golden fixtures never need to carry weights.

Key names and shapes follow the reference module tree:
  * TransformerLanguageModel.__init__  transformer_language_model.py:34-72
  * TransformerLayer.__init__          transformer_layer.py:6-29 (+ cross-attention setter :31-42)
  * Attention.__init__                 attention.py:12-49
  * Perceiver.__init__                 perceiver.py:6-29
  * TransformerVAE.__init__            transformer_vae.py:26-40
"""
from collections import OrderedDict
from dataclasses import dataclass
import hashlib

import numpy as np
import torch

VOCAB_SIZE = 2 ** 15  # transformer_language_model.py:13


@dataclass
class HParams:
    """The subset of TransformerVAEHparams the training step reads."""
    d_model: int = 512
    num_heads: int = 8
    num_layers: int = 6
    latent_depth: int = 64
    kl_weight: float = 1.0
    num_latents: int = 64          # transformer_vae.py:35 (hard-coded 64)
    vocab_size: int = VOCAB_SIZE
    attn_window: int = 0           # decoder: 0 = dense, else sparse_self_attention with attn_window_size

    @property
    def enc_layers(self) -> int:   # transformer_vae.py:35 -> Perceiver(num_layers // 2)
        return self.num_layers // 2

    @property
    def enc_heads(self) -> int:    # perceiver.py:13
        return self.d_model // 64


def _attention_params(prefix, d, learned_queries):
    out = OrderedDict()
    if learned_queries:
        out[prefix + 'learned_queries'] = (1, learned_queries, d)
    else:
        out[prefix + 'q_linear.weight'] = (d, d)
        out[prefix + 'q_linear.bias'] = (d,)
    for name in ('k_linear', 'v_linear', 'output_linear', 'pos_linear'):
        out[prefix + name + '.weight'] = (d, d)
        out[prefix + name + '.bias'] = (d,)
    return out


def _layer_params(prefix, d, learned_queries=None, cross=False):
    out = _attention_params(prefix + 'attention.', d, learned_queries)
    out[prefix + 'ffn.0.weight'] = (4 * d, d)
    out[prefix + 'ffn.0.bias'] = (4 * d,)
    out[prefix + 'ffn.2.weight'] = (d, 4 * d)
    for ln in ('attn_layer_norm', 'ffn_layer_norm'):
        out[prefix + ln + '.weight'] = (d,)
        out[prefix + ln + '.bias'] = (d,)
    if cross:
        out.update(_attention_params(prefix + 'cross_attention.', d, None))
        for ln in ('cross_attn_layer_norm', 'context_layer_norm'):
            out[prefix + ln + '.weight'] = (d,)
            out[prefix + ln + '.bias'] = (d,)
    return out


def param_shapes(hp: HParams) -> 'OrderedDict[str, tuple]':
    """Unique parameters (tied weights listed once, as `input_layer.0.weight`), in the
    reference's `named_parameters()` order."""
    d, V = hp.d_model, hp.vocab_size
    assert hp.enc_layers > 1, 'perceiver.py:12 asserts num_layers > 1'
    out = OrderedDict()
    out['input_layer.0.weight'] = (V, d)
    out['output_layer.0.weight'] = (d, d)
    out['output_layer.0.bias'] = (d,)
    out['output_layer.2.weight'] = (d,)
    out['output_layer.2.bias'] = (d,)
    out['output_layer.3.bias'] = (V,)          # .3.weight is tied to input_layer.0.weight
    for i in range(hp.num_layers):
        out.update(_layer_params(f'decoder_layers.{i}.', d))
    out['q_of_z_given_x.linear.weight'] = (2 * hp.latent_depth, d)
    out['q_of_z_given_x.linear.bias'] = (2 * hp.latent_depth,)
    out.update(_layer_params('encoder.first_layer.', d, learned_queries=hp.num_latents))
    out.update(_layer_params('encoder.bottleneck.', d, learned_queries=1))
    for j in range(hp.enc_layers - 2):
        out.update(_layer_params(f'encoder.middle_layers.{j}.', d, cross=True))
    for i in range(hp.num_layers):
        out[f'z_projections.{i}.weight'] = (d, hp.latent_depth)
        out[f'z_projections.{i}.bias'] = (d,)
    return out


TIED_ALIASES = ('output_layer.3.weight', 'encoder_input_layer.0.weight')


# ---- portable counter-based generator: splitmix64 -> Box-Muller --------------------------------

_M64 = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(counter: np.ndarray) -> np.ndarray:
    z = counter + np.uint64(0x9E3779B97F4A7C15)
    z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def portable_normal(n: int, key: str, seed: int) -> np.ndarray:
    """n standard normals from (seed, key); identical on every machine with numpy."""
    base = int.from_bytes(hashlib.sha256(f'{seed}:{key}'.encode()).digest()[:8], 'little')
    half = (n + 1) // 2
    with np.errstate(over='ignore'):
        ctr = (np.arange(2 * half, dtype=np.uint64) + np.uint64(base)) & _M64
        bits = _splitmix64(ctr)
    u = ((bits >> np.uint64(11)).astype(np.float64) + 0.5) * (1.0 / 9007199254740992.0)
    u1, u2 = u[:half], u[half:]
    r = np.sqrt(-2.0 * np.log(u1))
    z = np.concatenate([r * np.cos(2 * np.pi * u2), r * np.sin(2 * np.pi * u2)])
    return z[:n]


def portable_ids(shape, seed: int, low: int = 3, high: int = VOCAB_SIZE) -> np.ndarray:
    """Synthetic token ids uniform in [low, high) with [CLS]=1 at position 0."""
    n = int(np.prod(shape))
    with np.errstate(over='ignore'):
        bits = _splitmix64((np.arange(n, dtype=np.uint64) + np.uint64(seed * 7919 + 11)) & _M64)
    ids = (low + (bits % np.uint64(high - low)).astype(np.int64)).reshape(shape)
    ids[..., 0] = 1
    return ids


def init_params(hp: HParams, seed: int = 0, test_init: bool = True) -> 'OrderedDict[str, torch.Tensor]':
    """Deterministic fp32 parameters.

    test_init=True perturbs biases and LayerNorm affine params away from 0/1 so the parity tests
    exercise every bias/affine path. test_init=False mirrors `initialize_weights`
    (language_model.py:80-96: N(0, 0.02) weights, zero biases, LN untouched) with learned queries
    ~ N(0,1) (attention.py:31)."""
    out = OrderedDict()
    for name, shape in param_shapes(hp).items():
        n = int(np.prod(shape))
        z = portable_normal(n, name, seed).reshape(shape)
        if name.endswith('learned_queries'):
            v = z
        elif 'layer_norm' in name or name.startswith('output_layer.2.'):
            if name.endswith('.weight'):
                v = 1.0 + 0.1 * z if test_init else np.ones(shape)
            else:
                v = 0.1 * z if test_init else np.zeros(shape)
        elif name.endswith('.bias'):
            v = 0.02 * z if test_init else np.zeros(shape)
        else:
            v = 0.02 * z
        out[name] = torch.from_numpy(np.ascontiguousarray(v, dtype=np.float32))
    return out
