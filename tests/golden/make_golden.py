"""Generate golden vectors by running the REAL reference (`/root/reference`) on CPU, fp32.

Run in the survey/build container only (the GPU box has no /root/reference):

    python tests/golden/make_golden.py

Writes tests/golden/<name>.npz (+ reference_keys.json). Weights are never stored: both the reference and
every consumer regenerate them from `oracle.params.init_params(hp, seed)` (portable splitmix64 normals).
Determinism controls: dropout p=0, `Normal.rsample` patched to use injected eps,
kl_weight pinned.
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

from oracle.params import HParams, init_params, portable_normal, portable_ids, TIED_ALIASES  # noqa: E402
import ref_stubs  # noqa: E402

# name -> (d_model, num_heads, num_layers, L, B, padded)
CONFIGS = {
    'tiny': (128, 8, 4, 128, 4, False),          # minimal buildable "tiny" (4 layers, decoder hd 16)
    'tiny_pad': (128, 8, 4, 128, 4, True),
    'small6_pad': (256, 4, 6, 192, 3, True),     # hd 64, one middle (cross-attention) encoder layer
    'hd96': (384, 4, 6, 128, 2, True),           # decoder hd 96, encoder 6 heads x 64
    'c2shape': (512, 8, 6, 512, 2, False),       # the C2 model at B=2
    'c4shape': (768, 8, 12, 1024, 2, True),      # the C4/C5 model (decoder hd 96, encoder 12 x 64) at L=1024, B=2
    'c5shape': (768, 8, 12, 2048, 2, True),      # the C5 sequence length (L=2048), second sequence padded
}
N_SAMPLE = 64   # gradient elements sampled per parameter


def lengths_for(B, L, padded):
    if not padded:
        return [L] * B
    return [L - (37 * b) % (L // 2) for b in range(B)]


def make_batch(B, L, padded, seed):
    ids = portable_ids((B, L), seed)
    lens = lengths_for(B, L, padded)
    for b, n in enumerate(lens):
        ids[b, n:] = 0
    return ids, np.asarray(lens, dtype=np.int64)


def sample_indices(n, key):
    z = portable_normal(N_SAMPLE, 'idx:' + key, 99)
    return (np.abs(z * 1e6).astype(np.int64) % n).astype(np.int64)


def run_config(sv, name, cfg, seed=1234):
    d, H, NL, L, B, padded = cfg
    hp = HParams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64, kl_weight=0.7)
    rhp = sv.TransformerVAEHparams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64,
                                   sparse_self_attention=False, kl_weight=0.7, start_token=1, end_token=2)
    torch.manual_seed(0)
    model = sv.TransformerVAE(rhp)
    params = init_params(hp, seed)
    sd = dict(params)
    for alias in TIED_ALIASES:
        sd[alias] = params['input_layer.0.weight']
    missing = set(model.state_dict().keys()) ^ set(sd.keys())
    assert not missing, missing
    model.load_state_dict(sd, strict=True)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0

    ids, lens = make_batch(B, L, padded, seed + 1)
    eps = torch.from_numpy(portable_normal(B * 64, 'eps', seed).reshape(B, 1, 64).astype(np.float32))
    eps10 = torch.from_numpy(portable_normal(10 * B * 64, 'eps10', seed).reshape(10, B, 1, 64).astype(np.float32))

    from torch.distributions import Normal

    def rsample(self, sample_shape=torch.Size()):
        e = eps if len(sample_shape) == 0 else eps10
        return self.loc + e * self.scale

    Normal.rsample = rsample
    PaddedTensor = sys.modules['sparse_vae.core.padded_tensor'].PaddedTensor
    batch = {
        'token_ids': PaddedTensor.from_raw(torch.from_numpy(ids.astype(np.int16))),
        'num_tokens': torch.from_numpy(lens),
        'num_bytes': torch.from_numpy(lens),
    }
    out = model.training_step(batch, 0)
    out['loss'].backward()

    rec = {
        'ids': ids.astype(np.int32), 'lens': lens, 'eps': eps.numpy(), 'eps10': eps10.numpy(),
        'cfg': np.asarray([d, H, NL, L, B, int(padded), seed], dtype=np.int64),
        'kl_weight': np.float64(0.7),
        'loss': np.float64(out['loss'].item()),
        'train_nll': np.float64(model.logged['train_nll'].item()),
        'train_kl': np.float64(model.logged['train_kl'].item()),
        'mutual_info': np.float64(model.logged['train_mc_mutual_info'].item()),
        'mu': out['posterior'].loc.numpy().reshape(B, 64),
        'scale': out['posterior'].scale.numpy().reshape(B, 64),
    }
    names = []
    for pname, prm in model.named_parameters():
        if prm.grad is None:
            continue
        names.append(pname)
        g = prm.grad.detach().flatten().double().numpy()
        rec['gnorm/' + pname] = np.float64(np.linalg.norm(g))
        idx = sample_indices(g.size, pname)
        rec['gidx/' + pname] = idx
        rec['gval/' + pname] = g[idx].astype(np.float32)
    rec['grad_names'] = np.asarray(names)

    with torch.no_grad():                         # argmax reconstructions at z = mu
        x = model.input_layer(batch['token_ids'].long())
        logits = model.reconstruct(x, out['posterior'].loc)[..., :-1, :]
        top2 = logits.topk(2, dim=-1)
        rec['argmax'] = top2.indices[..., 0].numpy().astype(np.int32)
        rec['margin'] = (top2.values[..., 0] - top2.values[..., 1]).numpy().astype(np.float32)
        rec['logit_rows'] = logits[0, [0, L // 2]].numpy().astype(np.float32)
    np.savez_compressed(os.path.join(HERE, name + '.npz'), **rec)
    print(f'{name}: loss={rec["loss"]:.6f} nll={rec["train_nll"]:.6f} kl={rec["train_kl"]:.6f} '
          f'grads={len(names)}')
    return model


def op_vectors(sv):
    core = sys.modules['sparse_vae.core.attention']
    rec = {}
    for i, (shape, start, max_pos) in enumerate([((2, 5, 16), 0, 10000), ((3, 7, 64), 3, 10000),
                                                  ((1, 300, 32), 0, 256)]):
        x = torch.from_numpy(portable_normal(int(np.prod(shape)), f'rot{i}', 5).reshape(shape).astype(np.float32))
        rec[f'rot{i}_in'] = x.numpy().copy()
        rec[f'rot{i}_meta'] = np.asarray([start, max_pos])
        rec[f'rot{i}_out'] = core.encode_position_rotary(x.clone(), start, max_pos=max_pos).numpy()

    # RAdam: 8 steps crosses the SGD-momentum (steps 1-4) -> rectified (>= 5) switch.
    RAdam = sys.modules['sparse_vae.core.rectified_adam'].RAdam
    p0 = torch.from_numpy(portable_normal(300, 'radam_p', 5).astype(np.float32)).reshape(10, 30)
    p1 = torch.from_numpy(portable_normal(7, 'radam_q', 5).astype(np.float32))
    prm = [torch.nn.Parameter(p0.clone()), torch.nn.Parameter(p1.clone())]
    opt = RAdam(prm, lr=3e-3, weight_decay=0.01)
    rec['radam_p0'], rec['radam_p1'] = p0.numpy(), p1.numpy()
    for s in range(8):
        g0 = portable_normal(300, f'radam_g0_{s}', 5).astype(np.float32).reshape(10, 30)
        g1 = portable_normal(7, f'radam_g1_{s}', 5).astype(np.float32)
        rec[f'radam_g0_{s}'], rec[f'radam_g1_{s}'] = g0, g1
        prm[0].grad, prm[1].grad = torch.from_numpy(g0), torch.from_numpy(g1)
        opt.step()
        rec[f'radam_out0_{s}'] = prm[0].detach().numpy().copy()
        rec[f'radam_out1_{s}'] = prm[1].detach().numpy().copy()

    lm = sys.modules['sparse_vae.core.language_model']
    rec['cosine'] = np.asarray([lm.cosine_decay(1000, s) for s in (0, 1, 250, 500, 999)])
    np.savez_compressed(os.path.join(HERE, 'ops.npz'), **rec)
    print('ops: written')


def sparse_vectors(sv):
    """The block layout of the reference's SparseAttention (sparse_attention.py:39-60) for several windows,
    and the attention module's sparse rotary base (attention.py:52). The Triton blocksparse kernels that
    consume the layout (GPU-only, triton 1.1) cannot run here: their softmax masking is parity-unpinned."""
    SA = sys.modules['sparse_vae.core.sparse_attention'].SparseAttention
    Att = sys.modules['sparse_vae.core.attention'].Attention
    rec = {}
    for w in (1, 2, 3, 4, 6):
        lay = SA(window_size=w, max_seq_len=640, num_heads=2).get_master_layout()
        rec[f'layout_w{w}'] = lay.numpy().astype(np.int8)
    for w in (4, 2):
        a = Att(64, 4, causal=True, sparse=w)
        rec[f'window_of_sparse_{w}'] = np.asarray([a.sparse_attention.window_size,
                                                   a.sparse_attention.block_size, a.sparse_attention.causal,
                                                   a.sparse_attention.include_cls])
    np.savez_compressed(os.path.join(HERE, 'sparse.npz'), **rec)
    print('sparse: written')


def _ref_model(sv, hp, seed, window=0, emb_scale=1.0):
    rhp = sv.TransformerVAEHparams(d_model=hp.d_model, num_heads=hp.num_heads, num_layers=hp.num_layers,
                                   latent_depth=64, sparse_self_attention=bool(window),
                                   attn_window_size=window or 4, kl_weight=1.0, start_token=1, end_token=2)
    torch.manual_seed(0)
    model = sv.TransformerVAE(rhp)
    params = init_params(hp, seed)
    params['input_layer.0.weight'] = params['input_layer.0.weight'] * emb_scale
    sd = dict(params)
    for alias in TIED_ALIASES:
        sd[alias] = params['input_layer.0.weight']
    model.load_state_dict(sd, strict=True)
    for m in model.modules():
        if isinstance(m, torch.nn.Dropout):
            m.p = 0.0
    model.eval()
    return model


# name -> (d_model, num_heads, num_layers, window, B, max_length, repetition_penalty, seed)
GEN_CONFIGS = {
    'gen_dense': (128, 8, 4, 0, 3, 48, 1.2, 31),
    'gen_dense_nopen': (128, 4, 4, 0, 2, 40, 1.0, 32),
    'gen_sparse': (128, 2, 4, 2, 2, 150, 1.2, 33),      # window 2: the KV cache shifts from position 96 on
}
EMB_SCALE = 10.0   # peaked logits (tied head): greedy top-1/top-2 margins far above fp32 rounding


def generation_vectors(sv):
    """TransformerVAE.sample (transformer_vae.py:95-128) greedy (temperature 0) with the KV cache
    (attention.py:107-168) and GenerationState (generation.py), dense and sliding-window. The end token is
    chosen from a first run (a token row 0 emits from step 5 on and no other row emits) so that early
    stopping is exercised while the other rows run to max_length (and through the sliding-window cache shift)."""
    for name, (d, H, NL, window, B, T, pen, seed) in GEN_CONFIGS.items():
        hp = HParams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64, kl_weight=1.0, attn_window=window)
        model = _ref_model(sv, hp, seed, window, EMB_SCALE)
        z = torch.from_numpy(portable_normal(B * 64, 'z', seed).reshape(B, 1, 64).astype(np.float32))
        with torch.no_grad():
            first = model.sample(T, B, z=z.clone(), temperature=0.0, repetition_penalty=pen)
            others = set(first[1:].flatten().tolist())
            k = next(i for i in range(4, T - 1) if int(first[0, i]) not in others)
            end = int(first[0, k])          # row 0 stops at step k + 1; every other row runs to max_length
            model.end_token = end
            out = model.sample(T, B, z=z.clone(), temperature=0.0, repetition_penalty=pen)
        rec = {'cfg': np.asarray([d, H, NL, window, B, T, seed], dtype=np.int64), 'penalty': np.float64(pen),
               'emb_scale': np.float64(EMB_SCALE), 'start_token': np.int64(1), 'end_token': np.int64(end),
               'z': z.numpy(), 'tokens': out.numpy().astype(np.int32), 'first_run': first.numpy().astype(np.int32)}
        np.savez_compressed(os.path.join(HERE, name + '.npz'), **rec)
        print(f'{name}: end={end} tokens[0,:12]={out[0, :12].tolist()}')


def iw_vectors(sv):
    """TransformerVAE.test_step (transformer_vae.py:71-79) -> estimate_log_prob_iw (continuous_autoencoder.py:
    62-80) with the rsample draws injected, for chunk size 1 (num_iter = num_samples, the reference's own
    100/100 setting) and chunk size = B (the reference's [chunk, B, 1] + [chunk, B] broadcasting)."""
    d, H, NL, L, B, seed = 128, 8, 4, 96, 3, 41
    hp = HParams(d_model=d, num_heads=H, num_layers=NL, latent_depth=64, kl_weight=1.0)
    model = _ref_model(sv, hp, seed)
    ids, lens = make_batch(B, L, True, seed + 1)
    PaddedTensor = sys.modules['sparse_vae.core.padded_tensor'].PaddedTensor
    from torch.distributions import Normal
    rec = {'ids': ids.astype(np.int32), 'lens': lens, 'cfg': np.asarray([d, H, NL, L, B, seed], dtype=np.int64)}
    for tag, S, n_iter in (('c1', 100, 100), ('cB', 6, 2)):
        eps = torch.from_numpy(portable_normal(S * B * 64, 'eps_iw_' + tag, seed).reshape(S, B, 1, 64)
                               .astype(np.float32))
        state = {'i': 0}

        def rsample(self, sample_shape=torch.Size()):
            c = int(sample_shape[0])
            e = eps[state['i']:state['i'] + c]
            state['i'] += c
            return self.loc + e * self.scale

        Normal.rsample = rsample
        batch = {'token_ids': PaddedTensor.from_raw(torch.from_numpy(ids.astype(np.int16))),
                 'num_tokens': torch.from_numpy(lens), 'num_bytes': torch.from_numpy(lens)}
        with torch.no_grad():
            if tag == 'c1':      # the reference's test_step: num_samples = num_iter = 100 (chunk 1)
                orig = type(model).estimate_log_prob_iw
                captured = {}

                def spy(self, *a, **k):
                    r = orig(self, *a, **k)
                    captured['log_prob'] = r.clone()
                    return r

                type(model).estimate_log_prob_iw = spy
                try:
                    nll_iw = model.test_step(batch, 0)
                finally:
                    type(model).estimate_log_prob_iw = orig
                log_prob = captured['log_prob']
                rec['nll_iw'] = np.float64(nll_iw.item())
            else:                # chunk = B: called directly (test_step hard-codes 100/100)
                original = batch['token_ids'].long()
                x = model.input_layer(original)
                posterior = model.q_of_z_given_x(model.encoder(x))
                log_prob = model.estimate_log_prob_iw(posterior, x, original, num_samples=S, num_iter=n_iter)
        assert state['i'] == S
        rec[f'eps_{tag}'] = eps.numpy()
        rec[f'num_iter_{tag}'] = np.int64(n_iter)
        rec[f'log_prob_{tag}'] = log_prob.numpy()
        print(f'iw {tag}: log_prob shape={tuple(log_prob.shape)} mean={log_prob.mean().item():.4f}')
    np.savez_compressed(os.path.join(HERE, 'iw.npz'), **rec)


# robust_cross_entropy's chunked branch (language_model.py:161-170): logits [33, 999, 32768] = 1.08e9 > 2^30
# elements -> cdiv = 2 chunks of 500 / 499 sequence positions, mean of the per-chunk means. The logits are the
# rank-2 product a (x) w + u (x) s with every factor bf16-representable, so a bf16-operand / f32-accumulate GEMM
# with K = 2 reproduces them bit for bit (each product is exact in f32, one rounding at the sum); only the factors
# and labels are stored. Padding lengths put most ignored positions into the second chunk, so the mean of means
# differs clearly from the single mean.
CE_SHAPE = (33, 999, 2 ** 15)


def ce_logits(a, u, w, s):
    logits = a[:, :, None] * w[None, None, :]
    logits.addcmul_(u[:, :, None], s[None, None, :])
    return logits


def ce_vectors(sv):
    lm = sys.modules['sparse_vae.core.language_model']
    import torch.nn.functional as F
    B, L1, V = CE_SHAPE

    def bf(x):
        return torch.from_numpy(np.asarray(x, dtype=np.float32)).bfloat16().float()

    a = bf(portable_normal(B * L1, 'ce_a', 7)).reshape(B, L1)
    u = bf(portable_normal(B * L1, 'ce_u', 7)).reshape(B, L1)
    w = bf(2.0 * portable_normal(V, 'ce_w', 7))
    s = bf(portable_normal(V, 'ce_s', 7))
    ids = portable_ids((B, L1 + 1), 71)
    lens = np.asarray([L1 + 1 - (37 * b) % 700 for b in range(B)], dtype=np.int64)
    for b, n in enumerate(lens):
        ids[b, n:] = 0
    labels = torch.from_numpy(ids[:, 1:].astype(np.int64))
    tok_w = torch.from_numpy(portable_ids((V,), 5, low=1, high=9).astype(np.float32))   # class weights 1..8
    tok_w[0] = 1.0
    logits = ce_logits(a, u, w, s)
    assert -(-logits.numel() // 2 ** 30) == 2
    with torch.no_grad():
        nll = lm.robust_cross_entropy(logits, labels)
        wnll = lm.robust_cross_entropy(logits, labels, weight=tok_w)
        single = F.cross_entropy(logits.flatten(end_dim=1), labels.flatten(), ignore_index=0)
    rec = {'a': a.numpy(), 'u': u.numpy(), 'w': w.numpy(), 's': s.numpy(), 'labels': labels.numpy().astype(np.int32),
           'lens': lens, 'tok_w': tok_w.numpy(), 'nll': np.float64(nll.item()), 'wnll': np.float64(wnll.item()),
           'single_mean': np.float64(single.item())}
    np.savez_compressed(os.path.join(HERE, 'ce_chunked.npz'), **rec)
    print(f'ce_chunked: nll={nll.item():.6f} weighted={wnll.item():.6f} single-chunk mean={single.item():.6f}')


def main():
    torch.set_num_threads(min(8, os.cpu_count()))
    sv = ref_stubs.import_reference()
    keys = {}
    only = sys.argv[1:]
    if only == ['sparse']:
        sparse_vectors(sv)
        return
    if only == ['ce']:
        ce_vectors(sv)
        return
    if only == ['eval']:
        generation_vectors(sv)
        iw_vectors(sv)
        return
    for name, cfg in CONFIGS.items():
        if only and name not in only:
            continue
        model = run_config(sv, name, cfg)
        keys[name] = {k: list(v.shape) for k, v in model.state_dict().items()}
    kpath = os.path.join(HERE, 'reference_keys.json')
    if only and os.path.exists(kpath):
        with open(kpath) as f:
            keys = {**json.load(f), **keys}
    with open(kpath, 'w') as f:
        json.dump(keys, f, indent=0)
    if not only:
        op_vectors(sv)


if __name__ == '__main__':
    main()
