"""robust_cross_entropy's chunked branch on the device (language_model.py:161-170): the vocabulary-head GEMM's
CE-statistics epilogue + ce_finalize / ce_weighted_nll / ce_grad with nchunks > 1.

* Against the REFERENCE's own values (tests/golden/ce_chunked.npz, made by make_golden.py ce): the fixture's
  logits [33, 999, 32768] (1.08e9 elements -> 2 chunks) are a rank-2 product of bf16-representable factors, so the
  head GEMM (bf16 operands, f32 accumulation, K = 512 with two non-zero columns) reproduces them exactly; nll and
  the class-weighted nll (val_bpb) within 1e-5 rel.
* dlogits for nchunks = 2 (the fixture's split) and 3 (forced) against torch fp32 autograd of the same chunked
  mean of means: 1e-2 rel (bf16 storage of the gradient); the output-bias gradient likewise.
"""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

from golden_util import ce_logits, setup_ce  # noqa: E402

if torch.cuda.is_available():
    from sparse_vae import kernels as K
    from sparse_vae import _native as N
    dev = torch.device('cuda')


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm()).item()


def _head_stats(t, labels, d=512):
    """Run the head GEMM on the fixture: rows = B * L (position L-1 of each sequence is the label-0 row the
    engine carries), hh[:, 0:2] = (a, u), W[:, 0:2] = (w, s), everything else 0, bias 0."""
    B, L1 = t['a'].shape
    L, V = L1 + 1, t['w'].numel()
    T = B * L
    hh = torch.zeros(B, L, d, device=dev)
    hh[:, :L1, 0] = t['a'].to(dev)
    hh[:, :L1, 1] = t['u'].to(dev)
    hh = hh.view(T, d).bfloat16()
    W = torch.zeros(V, d, device=dev)
    W[:, 0], W[:, 1] = t['w'].to(dev), t['s'].to(dev)
    W = W.bfloat16()
    lab = torch.zeros(B, L, dtype=torch.int32, device=dev)
    lab[:, :L1] = labels.to(dev)
    lab = lab.view(T)
    ntile = V // 128
    logits = torch.empty(T, V, dtype=torch.bfloat16, device=dev)
    part = torch.empty(T, ntile, 2, device=dev)
    ll = torch.zeros(T, device=dev)
    K.gemm(hh, W, logits, T, V, d, epi=N.EPI_CE_STATS, bias=torch.zeros(V, device=dev), aux=part, labels=lab,
           label_logit=ll)
    return B, L, V, T, logits, part, ll, lab, ntile


def test_chunked_nll_matches_reference():
    g, t, labels = setup_ce()
    B, L, V, T, logits, part, ll, lab, ntile = _head_stats(t, labels)
    nchunks, chunk_len = K.ce_chunking(B, L, V)
    assert (nchunks, chunk_len) == (2, 500)
    lse, rl, cw, nll = (torch.empty(T, device=dev), torch.empty(T, device=dev), torch.empty(nchunks, device=dev),
                        torch.empty(1, device=dev))
    K.ce_finalize(part, ntile, ll, lab, T, L, nchunks, chunk_len, lse, rl, cw, nll)
    want = float(g['nll'])
    assert abs(nll.item() - want) / want < 1e-5, (nll.item(), want)
    wn = torch.empty(1, device=dev)
    K.ce_weighted_nll(rl, lab, t['tok_w'].to(dev), T, L, nchunks, chunk_len, wn)
    assert abs(wn.item() - float(g['wnll'])) / float(g['wnll']) < 1e-5, (wn.item(), float(g['wnll']))
    # the stored (bf16) logits are the fixture's: within one bf16 rounding of the f32 values, identical to their
    # bf16 rounding almost everywhere (the MFMA's f32 sum may differ in the last bit, flipping a bf16 tie)
    ref = ce_logits(t['a'][:2], t['u'][:2], t['w'], t['s'])
    got = logits.view(B, L, V)[:2, :L - 1].float().cpu()
    assert ((got - ref).abs() <= ref.abs() * 2.0 ** -8 + 1e-30).all()
    assert (got != ref.bfloat16().float()).float().mean().item() < 1e-3


@pytest.mark.parametrize('nchunks', [2, 3])
def test_chunked_grad_matches_autograd(nchunks):
    g, t, labels = setup_ce()
    B, L, V, T, logits, part, ll, lab, ntile = _head_stats(t, labels)
    chunk_len = -(-(L - 1) // nchunks)
    lse, rl, cw, nll = (torch.empty(T, device=dev), torch.empty(T, device=dev), torch.empty(nchunks, device=dev),
                        torch.empty(1, device=dev))
    K.ce_finalize(part, ntile, ll, lab, T, L, nchunks, chunk_len, lse, rl, cw, nll)
    gs = torch.full((1,), 0.75, device=dev)
    db = torch.zeros(V, device=dev)
    K.ce_grad(logits, V, lse, cw, lab, gs, T, V, L, nchunks, chunk_len, dbias=db)
    # torch fp32 reference on the device: mean over chunks of F.cross_entropy(ignore_index=0) per chunk
    ref = ce_logits(t['a'].to(dev), t['u'].to(dev), t['w'].to(dev), t['s'].to(dev)).requires_grad_()
    y = labels.to(dev)
    loss = torch.stack([F.cross_entropy(lc.flatten(end_dim=1), yc.flatten(), ignore_index=0)
                        for lc, yc in zip(ref.split(chunk_len, dim=1), y.split(chunk_len, dim=1))]).mean()
    assert abs(nll.item() - loss.item()) / loss.item() < 1e-5
    (loss * 0.75).backward()
    dl = logits.view(B, L, V)
    assert dl[:, L - 1].abs().max().item() == 0.0               # the label-0 row carries no gradient
    assert _rel(dl[:, :L - 1], ref.grad) < 1e-2
    assert _rel(db, ref.grad.sum((0, 1))) < 1e-2
