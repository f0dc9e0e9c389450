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


def _prob_head(hh, W, bias, lab, T, L, V, d, nchunks, chunk_len, g=0.75, sat=None):
    """The engine's P-head (svae.h): forward (label logits, CE_PROB GEMM, finalize) and backward (prep, dW GEMM
    with weighted row sums, ROWSCALE_GATHER dX GEMM, one-hot part through the fused embedding backward with
    zero upstream gradient). Returns nll, row_loss and the gradients (dhh bf16, dW f32, dbias f32)."""
    ntile = V // 128
    coff = torch.empty(T, device=dev)
    K.ce_label_logit(hh, W, bias, lab, T, d, coff)
    Pm = torch.empty(T, V, dtype=torch.bfloat16, device=dev)
    part = torch.empty(ntile, T, device=dev)
    K.gemm(hh, W, Pm, T, V, d, epi=N.EPI_CE_PROB, bias=bias, aux=part, labels=lab, row_a=coff)
    lse, rl, cw, nll = (torch.empty(T, device=dev), torch.empty(T, device=dev), torch.empty(nchunks, device=dev),
                        torch.empty(1, device=dev))
    K.ce_prob_finalize(part, ntile, coff, lab, T, L, nchunks, chunk_len, lse, rl, cw, nll,
                       fix=None if sat is None else (hh, W, bias, Pm, sat))
    gs = torch.full((1,), g, device=dev)
    hh_r = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
    r, q = torch.empty(T, device=dev), torch.empty(T, device=dev)
    dbias, dW = torch.zeros(V, device=dev), torch.zeros(V, d, device=dev)
    K.ce_prob_bwd_prep(hh, lse, coff, cw, lab, gs, T, L, nchunks, chunk_len, d, hh_r, r, q, dbias)
    K.gemm(Pm, hh_r, dW, V, d, T, a_t=True, b_t=True, lda=V, ldb=d, ldc=d, epi=N.EPI_F32_ACC, a_rowsum=dbias,
           k_weight=r)
    dhh = torch.empty(T, d, dtype=torch.bfloat16, device=dev)
    K.gemm(Pm, W.t().contiguous(), dhh, T, d, V, epi=N.EPI_ROWSCALE_GATHER, labels=lab, row_a=r, row_b=q, gather=W,
           ldg=d)
    B = T // L
    ids = torch.zeros(B, L, dtype=torch.int32, device=dev)
    ids[:, 0] = 1
    ids[:, 1:] = lab.view(B, L)[:, :L - 1]
    K.embedding_bwd_ce(ids.view(T), torch.zeros(T, d, device=dev), dW, T, d, L, hh, q)
    return nll, rl, dhh, dW, dbias


def _torch_ref(hh, W, bias, lab, B, L, V, chunk_len, g=0.75):
    hr = hh.float().requires_grad_()
    Wr = W.float().requires_grad_()
    br = bias.clone().requires_grad_()
    logits = (hr @ Wr.t() + br).view(B, L, V)[:, :L - 1]
    y = lab.view(B, L)[:, :L - 1].long()
    loss = torch.stack([F.cross_entropy(lc.flatten(end_dim=1), yc.flatten(), ignore_index=0)
                        for lc, yc in zip(logits.split(chunk_len, dim=1), y.split(chunk_len, dim=1))]).mean()
    (loss * g).backward()
    return loss, hr.grad, Wr.grad, br.grad


def test_prob_head_chunked_matches_reference():
    """The P-head training path on the reference's chunked fixture: nll and val_bpb's weighted nll against the
    reference's values (1e-5), gradients against torch fp32 autograd (1e-2 rel)."""
    g, t, labels = setup_ce()
    B, L1 = t['a'].shape
    L, V, d = L1 + 1, t['w'].numel(), 512
    T = B * L
    hh = torch.zeros(B, L, d, device=dev)
    hh[:, :L1, 0], hh[:, :L1, 1] = t['a'].to(dev), t['u'].to(dev)
    hh = hh.view(T, d).bfloat16()
    W = torch.zeros(V, d, device=dev)
    W[:, 0], W[:, 1] = t['w'].to(dev), t['s'].to(dev)
    W = W.bfloat16()
    lab = torch.zeros(B, L, dtype=torch.int32, device=dev)
    lab[:, :L1] = labels.to(dev)
    lab = lab.view(T)
    bias = torch.zeros(V, device=dev)
    nchunks, chunk_len = K.ce_chunking(B, L, V)
    nll, rl, dhh, dW, dbias = _prob_head(hh, W, bias, lab, T, L, V, d, nchunks, chunk_len)
    assert abs(nll.item() - float(g['nll'])) / float(g['nll']) < 1e-5, (nll.item(), float(g['nll']))
    wn = torch.empty(1, device=dev)
    K.ce_weighted_nll(rl, lab, t['tok_w'].to(dev), T, L, nchunks, chunk_len, wn)
    assert abs(wn.item() - float(g['wnll'])) / float(g['wnll']) < 1e-5, (wn.item(), float(g['wnll']))
    loss, gh, gW, gb = _torch_ref(hh, W, bias, lab, B, L, V, chunk_len)
    assert abs(loss.item() - float(g['nll'])) / float(g['nll']) < 1e-5
    assert _rel(dhh[:, :2], gh[:, :2]) < 1e-2 and dhh[:, 2:].abs().max().item() == 0.0
    assert _rel(dW[:, :2], gW[:, :2]) < 1e-2
    assert _rel(dbias, gb) < 1e-2


@pytest.mark.parametrize('nchunks', [1, 3])
def test_prob_head_random_matches_autograd(nchunks):
    """P-head on unstructured operands (random hh, W, bias; padded rows; d = 256): nll 1e-5, dhh / dW / dbias
    1e-2 rel against torch fp32 autograd, with 1 and 3 sequence chunks."""
    torch.manual_seed(11 + nchunks)
    B, L, V, d = 8, 512, 32768, 256
    T = B * L
    hh = torch.randn(T, d, device=dev).bfloat16()
    W = (0.1 * torch.randn(V, d, device=dev)).bfloat16()
    bias = 0.5 * torch.randn(V, device=dev)
    lab = torch.randint(3, V, (B, L), dtype=torch.int32, device=dev)
    lab[:, -1] = 0
    lab[2, 300:] = 0                          # padded sequences
    lab[5, 100:] = 0
    lab = lab.view(T)
    chunk_len = -(-(L - 1) // nchunks)
    nll, rl, dhh, dW, dbias = _prob_head(hh, W, bias, lab, T, L, V, d, nchunks, chunk_len)
    loss, gh, gW, gb = _torch_ref(hh, W, bias, lab, B, L, V, chunk_len)
    assert abs(nll.item() - loss.item()) / loss.item() < 1e-5, (nll.item(), loss.item())
    assert _rel(dhh, gh) < 1e-2
    assert _rel(dW, gW) < 1e-2
    assert _rel(dbias, gb) < 1e-2


def test_prob_head_saturated_rows_are_recomputed():
    """rows whose largest logit is > 88 nats above the label logit saturate the CE_PROB epilogue's
    exponent (2^127). ce_prob_finalize_fix lists them and recomputes P, lse and the offset exactly, so nll and every
    gradient still match torch fp32 autograd (which, like the reference's fp32 log-softmax, is stable there)."""
    torch.manual_seed(5)
    B, L, V, d = 8, 512, 32768, 256
    T = B * L
    hh = torch.randn(T, d, device=dev)
    W = 0.1 * torch.randn(V, d, device=dev)
    W[777] = 0.0
    W[777, 0] = 1.0
    hot = [10, 20, 3000]
    for r in hot:
        hh[r] = 0.0
        hh[r, 0] = 150.0                 # logit of column 777: 150; every other logit within 15 of 0
    hh, W = hh.bfloat16(), W.bfloat16()
    bias = 0.5 * torch.randn(V, device=dev)
    lab = torch.randint(3, V, (B, L), dtype=torch.int32, device=dev)
    lab[lab == 777] = 778
    lab[:, -1] = 0
    lab = lab.view(T)
    chunk_len = L - 1
    sat = torch.empty(T + 1, dtype=torch.int32, device=dev)
    nll, rl, dhh, dW, dbias = _prob_head(hh, W, bias, lab, T, L, V, d, 1, chunk_len, sat=sat)
    assert sat[0].item() == len(hot)
    assert sorted(sat[1:1 + len(hot)].tolist()) == hot
    loss, gh, gW, gb = _torch_ref(hh, W, bias, lab, B, L, V, chunk_len)
    assert abs(nll.item() - loss.item()) / loss.item() < 1e-5, (nll.item(), loss.item())
    rows = torch.tensor(hot, device=dev)
    ref_rows = torch.logsumexp(hh[rows].float() @ W.float().t() + bias, -1) - (
        (hh[rows].float() * W[lab[rows].long()].float()).sum(-1) + bias[lab[rows].long()])
    torch.testing.assert_close(rl[rows], ref_rows, rtol=1e-5, atol=1e-3)
    assert _rel(dhh, gh) < 1e-2
    assert _rel(dW, gW) < 1e-2
    assert _rel(dbias, gb) < 1e-2
    # without the fix-up the same rows come out clipped (the check above is not vacuous)
    nll0, rl0, *_ = _prob_head(hh, W, bias, lab, T, L, V, d, 1, chunk_len)
    assert (rl0[rows] - ref_rows).abs().min().item() > 1.0
