"""ORACLE — test infrastructure only (see oracle/__init__.py).

CPU fp32 restatement of the reference TransformerVAE training hot path, written from the
reference's behaviour (file:line cited per function), functional over a parameter dict whose
keys are the reference `state_dict` keys (oracle/params.py).

Padding semantics of the reference's PaddedTensor (padded_tensor.py:54-69) are restated
explicitly: the token mask `pad = ids == 0` ([B, L]) reaches an attention call iff the KEY
sequence length equals L (the getter returns None on a length mismatch, :68-69).
"""
import math
from typing import Dict, Optional

import torch
import torch.nn.functional as F

__all__ = [
    'rotary', 'sparse_layout', 'sparse_mask', 'attention', 'transformer_layer', 'perceiver', 'conditional_gaussian',
    'sample_z', 'reconstruct', 'output_layer', 'robust_cross_entropy', 'marginal_kl',
    'training_step', 'radam_step', 'clip_grad_norm', 'cosine_decay', 'kl_anneal',
    'RAdamState', 'prior_log_prob', 'p_of_x_given_z', 'estimate_log_prob_iw', 'test_step_iw', 'generate',
]


def rotary(x: torch.Tensor, start: int = 0, max_pos: int = 10000) -> torch.Tensor:
    """encode_position_rotary, attention.py:194-208. Interleaved pairs (2i, 2i+1) over the FULL
    last dim, angles computed in x.dtype; (a, b) -> (a cos + (-b) sin, b cos + a sin)."""
    half = x.shape[-1] // 2
    freqs = torch.arange(half, dtype=x.dtype)
    pos = torch.arange(start, start + x.shape[-2], dtype=x.dtype)
    theta = max_pos ** (-freqs / half)
    ang = pos[:, None] * theta
    c, s = ang.cos(), ang.sin()
    a, b = x[..., 0::2], x[..., 1::2]
    out0 = a * c + (-b) * s
    out1 = b * c + a * s
    return torch.stack([out0, out1], dim=-1).flatten(-2)


def _linear(p, name, x, bias=True):
    return F.linear(x, p[name + '.weight'], p[name + '.bias'] if bias else None)


def sparse_layout(num_blocks: int, window: int) -> torch.Tensor:
    """SparseAttention.get_master_layout, sparse_attention.py:39-60, causal with include_cls: block row r
    attends block columns r - (window - 1) .. r (left_context = window, right_context = 0) and column 0."""
    r = torch.arange(num_blocks)
    off = r[:, None] - r[None, :]
    layout = (off >= 0) & (off < window)
    layout[:, 0] = True
    return layout


def sparse_mask(L: int, window: int) -> torch.Tensor:
    """[L, L] True where a key is NOT visible to a query under SparseAttention.__call__ (sparse_attention.py:
    75-92): outside the block layout, or above the diagonal (blocksparse softmax is_causal). Absent blocks
    never enter the softmax; the -1e7 shift below gives them exactly zero weight, so the two agree.
    For L % 32 != 0 (decoding prefixes) this is the key set the windowed KV cache of attention.py:107-140
    returns: the [CLS] block, the window - 1 previous blocks and the current block up to the query."""
    if L % 32 == 0:
        blk = sparse_layout(L // 32, window).repeat_interleave(32, 0).repeat_interleave(32, 1)
    else:
        b = torch.arange(L) // 32
        off = b[:, None] - b[None, :]
        blk = ((off >= 0) & (off < window)) | (b[None, :] == 0)
    return ~blk | torch.ones(L, L, dtype=torch.bool).triu(1)


def attention(p: Dict[str, torch.Tensor], pre: str, q_in, k_in, v_in, pad: Optional[torch.Tensor],
              num_heads: int, causal: bool = False, window: int = 0) -> torch.Tensor:
    """Attention.forward, attention.py:51-105: the dense branch, and with window > 0 the SparseAttention
    branch (:78-81; sparse_attention.py:75-92) restated densely with its block mask and rotary base
    max_pos = 2 * window * block_size (:52)."""
    B = k_in.shape[0]
    max_pos = 2 * window * 32 if window else 10000       # :52
    lq = p.get(pre + 'learned_queries')
    if lq is not None:                                   # :55-56
        q = lq.expand(B, *lq.shape[1:])
    else:                                                # :60-61
        q = rotary(_linear(p, pre + 'q_linear', q_in), max_pos=max_pos)
    k = rotary(_linear(p, pre + 'k_linear', k_in), max_pos=max_pos)       # :67, :70
    v = _linear(p, pre + 'v_linear', v_in)
    mask = pad if (pad is not None and pad.shape[-1] == k.shape[-2]) else None   # :75 + getter
    d = q.shape[-1]
    hd = d // num_heads

    def split(t):                                        # :76 '... l (h d) -> ... h l d'
        return t.reshape(t.shape[0], t.shape[1], num_heads, hd).transpose(1, 2)

    q, k, v = split(q), split(k), split(v)
    scores = q @ k.transpose(-1, -2) * k.shape[-1] ** -0.5          # :83
    causal_mask = None
    if window:                                           # sparse: band + [CLS] block + causal (is_causal)
        assert causal
        causal_mask = sparse_mask(q.shape[-2], window)
    elif causal:                                         # :85-87
        ql = q.shape[-2]
        causal_mask = torch.ones(ql, ql, dtype=torch.bool).triu(1)
    if mask is not None:                                 # :93
        mask = mask[..., None, None, :]
    if causal_mask is not None:                          # :94-95
        mask = mask | causal_mask if mask is not None else causal_mask
    if mask is not None:                                 # :97-98
        scores = scores - mask * 1e7
    out = scores.softmax(dim=-1) @ v                     # :100
    out = out.transpose(1, 2).reshape(out.shape[0], -1, d)            # :102
    return _linear(p, pre + 'output_linear', out)        # :103


def _ln(p, name, x):
    return F.layer_norm(x, (x.shape[-1],), p[name + '.weight'], p[name + '.bias'], 1e-5)


def transformer_layer(p, pre, x, pad, num_heads, causal=False, context=None,
                      dropout_mask: Optional[torch.Tensor] = None, dropout_p: float = 0.1, window: int = 0):
    """TransformerLayer.forward, transformer_layer.py:44-61 (pre-LN). `dropout_mask`, if given,
    is the keep-mask of nn.Dropout(0.1) at :58 (None = dropout disabled)."""
    y = _ln(p, pre + 'attn_layer_norm', x)
    y = attention(p, pre + 'attention.', y, y, y, pad, num_heads, causal, window)
    x = x + y if x.shape == y.shape else y               # :49
    if (pre + 'cross_attention.k_linear.weight') in p and context is not None:   # :51-54
        ctx = _ln(p, pre + 'context_layer_norm', context)
        y = _ln(p, pre + 'cross_attn_layer_norm', x)
        y = attention(p, pre + 'cross_attention.', y, ctx, ctx, pad, num_heads)
        x = x + y
    y = _ln(p, pre + 'ffn_layer_norm', x)                # :56-57
    y = F.linear(F.gelu(_linear(p, pre + 'ffn.0', y)), p[pre + 'ffn.2.weight'])
    if dropout_mask is not None:                         # :58
        y = y * dropout_mask / (1.0 - dropout_p)
    return x + y


def perceiver(p, x, pad, hp, dropout_masks=None):
    """Perceiver.forward, perceiver.py:39-50: first (64 learned queries) -> middle (self + cross)
    -> bottleneck (1 learned query). Heads = d_model // 64 (:13)."""
    h = hp.enc_heads
    dm = dropout_masks or {}
    z = transformer_layer(p, 'encoder.first_layer.', x, pad, h, dropout_mask=dm.get('encoder.first_layer'))
    for j in range(hp.enc_layers - 2):
        name = f'encoder.middle_layers.{j}'
        z = transformer_layer(p, name + '.', z, pad, h, context=x, dropout_mask=dm.get(name))
    return transformer_layer(p, 'encoder.bottleneck.', z, pad, h, dropout_mask=dm.get('encoder.bottleneck'))


def conditional_gaussian(p, h):
    """ConditionalGaussian.forward(get_kl=True), conditional_gaussian.py:18-28."""
    mu, logvar = _linear(p, 'q_of_z_given_x.linear', h).chunk(2, dim=-1)
    var = logvar.exp()
    scale = var.sqrt()
    kl = 0.5 * (mu ** 2 + var - logvar - 1.0)
    return mu, logvar, scale, kl


def sample_z(p, h, num_tokens, eps):
    """ContinuousVAE.sample_z, continuous_autoencoder.py:42-52 (rsample = loc + eps * scale)."""
    mu, logvar, scale, kl = conditional_gaussian(p, h)
    z = mu + eps * scale
    raw_kl = kl.flatten(1).sum(dim=-1)
    kl_mean = raw_kl.div(num_tokens).mean()
    return z, kl_mean, raw_kl, mu, logvar, scale


def output_layer(p, x):
    """output_layer, transformer_language_model.py:55-63 (Linear, GELU, LayerNorm, tied Linear)."""
    y = F.gelu(_linear(p, 'output_layer.0', x))
    y = _ln(p, 'output_layer.2', y)
    return F.linear(y, p['input_layer.0.weight'], p['output_layer.3.bias'])


def reconstruct(p, x, z, pad, hp, dropout_masks=None):
    """TransformerVAE.reconstruct, transformer_vae.py:85-93: position 0 of the residual stream is
    replaced by z_projections[i](z) before EVERY decoder layer."""
    dm = dropout_masks or {}
    for i in range(hp.num_layers):
        zh = _linear(p, f'z_projections.{i}', z)
        x = torch.cat([zh, x[..., 1:, :]], dim=-2)
        x = transformer_layer(p, f'decoder_layers.{i}.', x, pad, hp.num_heads, causal=True,
                              dropout_mask=dm.get(f'decoder_layers.{i}'), window=getattr(hp, 'attn_window', 0))
    return output_layer(p, x)


def robust_cross_entropy(logits, labels, weight=None, chunk_numel=2 ** 30):
    """language_model.py:161-170: one F.cross_entropy(ignore_index=0) when numel <= 2**30, else the
    mean of per-sequence-chunk means (torch.chunk along the sequence dim). `weight`: F.cross_entropy's class
    weights (the val_bpb metric passes the per-token byte counts, language_model.py:106-110). `chunk_numel`
    lowers the reference's 2**30 threshold for tests (the chunked branch at small shapes)."""
    chunks = -(-logits.numel() // chunk_numel)
    if chunks == 1:
        return F.cross_entropy(logits.flatten(end_dim=1), labels.flatten(), ignore_index=0, weight=weight)
    return torch.stack([
        F.cross_entropy(lc.flatten(end_dim=1), yc.flatten(), ignore_index=0, weight=weight)
        for lc, yc in zip(logits.chunk(chunks, dim=-2), labels.chunk(chunks, dim=-1))
    ]).mean()


def marginal_kl(mu, scale, eps_samples):
    """math_utils.py:51-58 with the 10 rsample draws injected (eps_samples [10, *mu.shape])."""
    samples = mu + eps_samples * scale
    x = samples[:, :, None]
    var = scale ** 2
    log_prob = -((x - mu) ** 2) / (2 * var) - scale.log() - math.log(math.sqrt(2 * math.pi))
    cross = log_prob.sum(dim=-1)
    marginal = cross.logsumexp(dim=2) - math.log(samples.shape[1])
    sample_prob = -0.5 * (samples.pow(2.0).sum(dim=-1).mean() + samples.shape[-1] * math.log(2 * math.pi))
    return sample_prob - marginal.mean()


def training_step(p, hp, ids, num_tokens, eps, kl_weight=None, eps_marginal=None,
                  pad: Optional[torch.Tensor] = 'auto', dropout_masks=None, ce_chunk_numel=2 ** 30):
    """TransformerVAE.training_step, transformer_vae.py:42-66 (stage='train').

    ids: int64 [B, L]; pad: [B, L] bool key-padding mask ('auto' = ids == 0, as PaddedTensor.from_raw
    does at padded_tensor.py:13-17; None = plain tensor, no mask). Returns the loss and the values the
    reference logs."""
    if isinstance(pad, str):
        pad = ids.eq(0)
    kl_weight = hp.kl_weight if kl_weight is None else kl_weight
    x = F.embedding(ids, p['input_layer.0.weight'])                       # :45
    enc = perceiver(p, x, pad, hp, dropout_masks)                          # :46
    z, kl, raw_kl, mu, logvar, scale = sample_z(p, enc, num_tokens, eps)   # :48
    logits = reconstruct(p, x, z, pad, hp, dropout_masks)[..., :-1, :]     # :50
    nll = robust_cross_entropy(logits, ids[..., 1:], chunk_numel=ce_chunk_numel)   # :51
    loss = nll + kl_weight * kl                                            # :55
    out = dict(loss=loss, nll=nll, kl=kl, raw_kl=raw_kl, train_kl=raw_kl.mean(),
               mu=mu, logvar=logvar, z=z, logits=logits)
    if ids.shape[0] > 1 and eps_marginal is not None:                      # :59-61
        out['mutual_info'] = kl - marginal_kl(mu, scale, eps_marginal)
    return out


# ---- host-side step pieces -----------------------------------------------------------------------

def clip_grad_norm(grads, max_norm):
    """torch.nn.utils.clip_grad_norm_ as called at language_model.py:120-122 (2-norm)."""
    norms = torch.stack([g.detach().double().norm() for g in grads])
    total = norms.norm()
    coef = torch.clamp(max_norm / (total + 1e-6), max=1.0)
    return total, [g * coef.to(g.dtype) for g in grads]


class RAdamState:
    def __init__(self):
        self.step = 1
        self.exp_avg = {}
        self.exp_avg_sq = {}


def radam_step(params, grads, state: RAdamState, lr, betas=(0.9, 0.999), eps=1e-6, weight_decay=0.01):
    """RAdam.step (lamb=False), rectified_adam.py:16-88. 1-indexed step; variance rectification when
    rho_t > 4, SGD-momentum update otherwise; decoupled weight decay. Returns new params."""
    beta1, beta2 = betas
    step = state.step
    beta2_t = beta2 ** step
    bcv = (1 - beta2_t) ** 0.5
    rho_inf = 2.0 / (1.0 - beta2) - 1.0
    rho_t = rho_inf - 2 * step * beta2_t / (1 - beta2_t)
    if rho_t > 4:
        r_t = (((rho_t - 4.0) * (rho_t - 2.0) * rho_inf) / ((rho_inf - 4.0) * (rho_inf - 2.0) * rho_t)) ** 0.5
        lr = lr * (r_t * bcv)
    bcm = 1 - beta1 ** step
    out = {}
    for name, prm in params.items():
        g = grads.get(name)
        if g is None:
            out[name] = prm
            continue
        m = state.exp_avg.get(name, torch.zeros_like(prm))
        v = state.exp_avg_sq.get(name, torch.zeros_like(prm))
        m = m * beta1 + g * (1 - beta1)
        v = v * beta2 + g * g * (1 - beta2)
        state.exp_avg[name], state.exp_avg_sq[name] = m, v
        prm = prm * (1 - lr * weight_decay)
        if rho_t > 4:
            denom = v.sqrt() / bcv + eps
            prm = prm - (lr / bcm) * (m / denom)
        else:
            prm = prm - (lr / bcm) * m
        out[name] = prm
    state.step += 1
    return out


def cosine_decay(decay_steps: int, cur_step: int) -> float:
    """language_model.py:135-141 (raises KeyboardInterrupt once fully decayed)."""
    progress = cur_step / max(1, decay_steps)
    if progress >= 1.0:
        raise KeyboardInterrupt
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * progress)))


def kl_anneal(kl_weight, kl_start, kl_end, max_steps, cur_step):
    """ContinuousVAE.on_after_backward, continuous_autoencoder.py:28-39."""
    if not max_steps or kl_weight >= kl_end:
        return kl_weight
    return kl_start + (kl_end - kl_start) * (cur_step / max_steps)


# ---- evaluation (importance-weighted NLL) and generation --------------------------------------------

def prior_log_prob(z):
    """ContinuousVAE.prior_log_prob, continuous_autoencoder.py:55-57."""
    return -0.5 * z.pow(2.0).sum(dim=-1) - math.log(math.sqrt(2 * math.pi)) * z.shape[-1]


def p_of_x_given_z(p, hp, x, z, labels, pad):
    """continuous_autoencoder.py:82-88: log p(x|z) summed over the sequence. x [c, B, L, d] (the expanded
    embedding), z [c, B, 1, Z], labels [c, B, L-1]; log_softmax column 0 zeroed, so label 0 adds 0."""
    c, B, L, d = x.shape
    xf, zf = x.reshape(c * B, L, d), z.reshape(c * B, 1, z.shape[-1])
    padf = pad.expand(c, B, L).reshape(c * B, L) if pad is not None else None
    logits = reconstruct(p, xf, zf, padf, hp)[..., :-1, :]
    log_probs = logits.log_softmax(dim=-1)
    log_probs[..., 0] = 0.0
    lp = log_probs.gather(dim=-1, index=labels.reshape(c * B, L - 1).unsqueeze(-1)).squeeze(-1).sum(dim=-1)
    return lp.reshape(c, B)


def estimate_log_prob_iw(p, hp, mu, scale, x, labels, pad, eps, num_iter):
    """ContinuousVAE.estimate_log_prob_iw, continuous_autoencoder.py:62-80, with the rsample draws injected:
    eps [num_samples, B, 1, Z] (chunk i uses eps[i*chunk:(i+1)*chunk]). The tensor shapes are the reference's
    own, so its broadcasting ([chunk, B, 1] + [chunk, B]) is reproduced as is."""
    S = eps.shape[0]
    assert S % num_iter == 0
    chunk = S // num_iter
    log_ws = []
    for it in range(num_iter):
        z = mu + eps[it * chunk:(it + 1) * chunk] * scale                   # [chunk, B, 1, Z]
        log_p_of_z = prior_log_prob(z)                                      # [chunk, B, 1]
        log_q_of_z = torch.distributions.Normal(mu, scale).log_prob(z).sum(dim=-1)
        lpx = p_of_x_given_z(p, hp, x.unsqueeze(0).expand(chunk, *x.shape), z,
                             labels.expand(chunk, *labels.shape)[..., 1:], pad)
        log_ws.append(log_p_of_z + lpx - log_q_of_z)
    return torch.cat(log_ws).logsumexp(dim=0) - math.log(S)


def test_step_iw(p, hp, ids, num_tokens, eps, num_iter, pad='auto'):
    """TransformerVAE.test_step, transformer_vae.py:71-79 (num_samples = eps.shape[0]). Returns nll_iw."""
    if isinstance(pad, str):
        pad = ids.eq(0)
    x = F.embedding(ids, p['input_layer.0.weight'])
    enc = perceiver(p, x, pad, hp)
    mu, logvar, scale, _ = conditional_gaussian(p, enc)
    log_prob = estimate_log_prob_iw(p, hp, mu, scale, x, ids, pad, eps, num_iter) / num_tokens
    return -log_prob.mean()


def generate(p, hp, z, max_length, start_token, end_token, repetition_penalty=1.2):
    """TransformerVAE.sample (transformer_vae.py:95-128) with GenerationState (generation.py) in its greedy
    branch (temperature <= 0 or top_k == 1), restated without a KV cache: each step recomputes the decoder
    over the prefix (position 0 replaced by z_projections[i](z) in every layer, as at step 1 of the cached
    decode) and reads the last position. Sparse attention: the windowed cache's key set (sparse_mask)."""
    B = z.shape[0]
    out = torch.zeros(B, max_length, dtype=torch.long)
    out[:, 0] = start_token
    live = torch.ones(B, dtype=torch.bool)
    idx = 1
    while not (idx >= max_length - 1 or not live.any()):                  # generation.py:83-84
        prefix = out[live, :idx]
        x = F.embedding(prefix, p['input_layer.0.weight'])
        logits = reconstruct(p, x, z[live].reshape(-1, 1, z.shape[-1]), None, hp)[:, -1]
        if repetition_penalty > 1.0:                                        # generation.py:35-41
            prev = out[live, max(idx - 512, 0):idx]
            pl = logits.gather(-1, prev)
            logits = logits.scatter(-1, prev, torch.where(pl < 0.0, pl * repetition_penalty,
                                                          pl / repetition_penalty))
        tok = logits.argmax(dim=-1)                                         # :44-45
        out[live, idx] = tok
        idx += 1
        cont = (tok != end_token) & (idx < max_length)                      # :73-75
        live[live.clone()] &= cont
    return out[:, 1:]
