"""Per-kernel numerics of libsvae.so against plain PyTorch fp32 references of the same ops (GPU only)."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

if torch.cuda.is_available():
    from sparse_vae import kernels as K
    from sparse_vae import _native as N
    from sparse_vae.engine import rotary_table
    import oracle

dev = 'cuda'


def _rel(a, b):
    return ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize('M,Nn,Kk', [(128, 128, 64), (200, 136, 72), (512, 384, 1024), (64, 1536, 512),
                                     (4000, 3064, 520)])   # last: >= 192 256x256 tiles -> gemm256 for a_t = 0
@pytest.mark.parametrize('a_t,b_t', [(0, 0), (0, 1), (1, 1), (1, 0)])
def test_gemm_layouts_exact(M, Nn, Kk, a_t, b_t):
    g = torch.Generator(device=dev).manual_seed(M + Nn + Kk)
    A = torch.randint(-3, 4, (M, Kk), device=dev, generator=g).float()
    B = torch.randint(-3, 4, (Kk, Nn), device=dev, generator=g).float()
    As = (A.t() if a_t else A).contiguous().bfloat16()
    Bs = (B if b_t else B.t()).contiguous().bfloat16()
    C = torch.zeros(M, Nn, device=dev)
    K.gemm(As, Bs, C, M, Nn, Kk, a_t=bool(a_t), b_t=bool(b_t), epi=N.EPI_F32)
    torch.cuda.synchronize()
    assert torch.equal(C, A @ B)


def test_gemm_split_k_atomic_and_acc():
    A = torch.randint(-2, 3, (4096, 256), device=dev).float()
    B = torch.randint(-2, 3, (4096, 384), device=dev).float()
    C = torch.ones(256, 384, device=dev)
    rs = torch.full((256,), 2.0, device=dev)
    K.gemm(A.bfloat16(), B.bfloat16(), C, 256, 384, 4096, a_t=True, b_t=True, epi=N.EPI_F32_ATOMIC, splits=4,
           a_rowsum=rs)
    assert torch.equal(C, 1 + A.t() @ B)
    assert torch.equal(rs, 2 + A.sum(0))
    K.gemm(A.bfloat16(), B.bfloat16(), C, 256, 384, 4096, a_t=True, b_t=True, epi=N.EPI_F32_ACC)
    assert torch.equal(C, 1 + 2 * (A.t() @ B))


@pytest.mark.parametrize('Kk,Nn', [(2048, 776), (2056, 200)])
@pytest.mark.parametrize('b_t', [True, False])
def test_gemm256_at_rowsum_k_weight_exact(b_t, Kk, Nn):
    """a_t on the 256x256 kernel with both B layouts (the vocabulary head's dW: MN-contiguous B; or K-contiguous):
    f32 accumulate with plain and k-weighted row sums, bit-exact on integer data, repeated (the k-weighted sums once
    mismatched in a DMA-order experiment). N 776: 64 x 4 = 256 tiles, ragged N, each of the first two column tiles
    sums one k-step of every K-tile; N 200: one column tile summing both k-steps, and a K tail (2056 = 32 x 64 + 8)."""
    g = torch.Generator(device=dev).manual_seed(5)
    M = 16384
    A = torch.randint(-2, 3, (Kk, M), device=dev, generator=g).float()
    B = torch.randint(-2, 3, (Kk, Nn), device=dev, generator=g).float()
    kw = torch.randint(-2, 3, (Kk,), device=dev, generator=g).float()
    Bs = (B if b_t else B.t().contiguous()).bfloat16()
    ref_c = 1 + A.t() @ B
    for use_kw in (False, True, True, True, True):
        C = torch.ones(M, Nn, device=dev)
        rs = torch.full((M,), 3.0, device=dev)
        K.gemm(A.bfloat16(), Bs, C, M, Nn, Kk, a_t=True, b_t=b_t, ldb=Nn if b_t else Kk,
               epi=N.EPI_F32_ACC, a_rowsum=rs, k_weight=kw if use_kw else None)
        torch.cuda.synchronize()
        assert torch.equal(C, ref_c)
        ref = 3 + ((A * kw[:, None]).sum(0) if use_kw else A.sum(0))
        bad = (rs != ref).nonzero().flatten()
        assert bad.numel() == 0, (use_kw, bad[:16].tolist(), (rs - ref)[bad[:16]].tolist())


@pytest.mark.parametrize('splits', [2, 3])
def test_gemm256_k_weight_split_slab_exact(splits):
    """The k-weighted row sums in split-K slab mode (the vocabulary head's dW at C4 / C5: 384 tiles run as 2 x 384):
    each split stores its partial tile into aux, slab_reduce adds them into C, the row sums of every split's K range
    add into a_rowsum; bit-exact on integer data (ragged N, K not a multiple of splits x 64), repeated."""
    g = torch.Generator(device=dev).manual_seed(9)
    Kk, M, Nn = 4160, 16384, 776
    A = torch.randint(-2, 3, (Kk, M), device=dev, generator=g).float()
    B = torch.randint(-2, 3, (Kk, Nn), device=dev, generator=g).float()
    kw = torch.randint(-2, 3, (Kk,), device=dev, generator=g).float()
    slab = torch.empty(splits * M * Nn, device=dev)
    ref_c = 1 + A.t() @ B
    ref_rs = 3 + (A * kw[:, None]).sum(0)
    for _ in range(3):
        C = torch.ones(M, Nn, device=dev)
        rs = torch.full((M,), 3.0, device=dev)
        K.gemm(A.bfloat16(), B.bfloat16(), C, M, Nn, Kk, a_t=True, b_t=True, ldb=Nn, epi=N.EPI_F32_ATOMIC,
               splits=splits, aux=slab, a_rowsum=rs, k_weight=kw)
        torch.cuda.synchronize()
        assert torch.equal(C, ref_c)
        bad = (rs != ref_rs).nonzero().flatten()
        assert bad.numel() == 0, (bad[:16].tolist(), (rs - ref_rs)[bad[:16]].tolist())


def test_gemm256_split_k_rowsum_exact():
    """dW layout on the 256x256 kernel: split-K f32 atomics + fused bias-gradient row sums, and the
    unsplit f32 accumulate (the tied head's dW), all bit-exact on integer data."""
    g = torch.Generator(device=dev).manual_seed(11)
    Kk = 32768
    for M, Nn, splits, use_slab in [(1536, 512, 16, False), (4096, 768, 1, False), (1536, 512, 16, True),
                                    (1024, 512, 8, True)]:
        A = torch.randint(-2, 3, (Kk, M), device=dev, generator=g).float()
        B = torch.randint(-2, 3, (Kk, Nn), device=dev, generator=g).float()
        C = torch.ones(M, Nn, device=dev)
        rs = torch.full((M,), 3.0, device=dev)
        epi = N.EPI_F32_ATOMIC if splits > 1 else N.EPI_F32_ACC
        slab = torch.empty(splits, M, Nn, device=dev) if use_slab else None   # slab split-K (plain stores + reduce)
        K.gemm(A.bfloat16(), B.bfloat16(), C, M, Nn, Kk, a_t=True, b_t=True, epi=epi, splits=splits, a_rowsum=rs,
               aux=slab)
        torch.cuda.synchronize()
        assert torch.equal(C, 1 + A.t() @ B)
        assert torch.equal(rs, 3 + A.sum(0))


@pytest.mark.parametrize('shapes', [((2048, 512, True), (512, 2048, False), 32768),    # FFN pair (8 splits)
                                    ((512, 512, True), (1536, 512, True), 32768),     # out-proj + QKV (16 splits)
                                    ((512, 512, True), (1024, 520, True), 4104),      # ragged N / K tail
                                    ((512, 512, True), (1536, 512, False), 600),      # too short to split: apart
                                    ((512, 512, True, 4096), (1024, 512, True, 32768), None),    # C2 encoder pair:
                                    ((768, 768, True, 4096), (1536, 768, True, 65536), None)])   # unequal splits
def test_linear_dw_pair_exact(shapes):
    """Two weight gradients in one paired launch (svae_gemm_pair, split-K slabs) equal dY^T X (+ the bias row sums)
    exactly on integer data, each into its own destination; the two may run over different row counts (then each
    gets its own split count, kernels.pair_splits)."""
    s0, s1, rows = shapes
    specs = [(t[0], t[1], t[2], t[3] if len(t) > 3 else rows) for t in (s0, s1)]
    g = torch.Generator(device=dev).manual_seed(specs[0][0] + specs[1][1] + specs[1][3])
    jobs, refs = [], []
    for n_out, n_in, with_bias, rows in specs:
        dY = torch.randint(-2, 3, (rows, n_out), device=dev, generator=g).float()
        X = torch.randint(-2, 3, (rows, n_in), device=dev, generator=g).float()
        Wg = torch.full((n_out, n_in), 0.5, device=dev)
        bg = torch.full((n_out,), 1.5, device=dev) if with_bias else None
        jobs.append((dY.bfloat16(), X.bfloat16(), Wg, rows, n_out, n_in, None, None, bg))
        refs.append((0.5 + dY.t() @ X, 1.5 + dY.sum(0) if with_bias else None))
    K.linear_dw_pair(*jobs)
    torch.cuda.synchronize()
    for j, (w_ref, b_ref) in zip(jobs, refs):
        assert torch.equal(j[2], w_ref)
        if b_ref is not None:
            assert torch.equal(j[8], b_ref)


@pytest.mark.parametrize('M,Nn,Kk', [(300, 256, 192), (4000, 3072, 520)])   # small: 128-tile kernels; big: gemm256
def test_gemm_epilogues(M, Nn, Kk):
    torch.manual_seed(0)
    X = torch.randn(M, Kk, device=dev).bfloat16()
    W = (torch.randn(Nn, Kk, device=dev) * 0.1).bfloat16()
    b = torch.randn(Nn, device=dev)
    ref = X.float() @ W.float().t() + b
    C = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_BF16, bias=b)
    assert _rel(C, ref) < 4e-3
    # GELU: C = gelu(acc + b), aux = gelu'(acc + b) (erf-exact reference; epilogue erf error <= 1.5e-7)
    gp = torch.empty_like(C)
    K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_GELU, bias=b, aux=gp, ldaux=Nn)
    r = ref.clone().requires_grad_()
    F.gelu(r).backward(torch.ones_like(r))
    assert _rel(C, F.gelu(ref)) < 4e-3 and _rel(gp, r.grad) < 4e-3
    # GELU backward: C = acc * aux
    G = torch.empty_like(C)
    K.gemm(X, W, G, M, Nn, Kk, epi=N.EPI_GELU_BWD, aux=gp, ldaux=Nn)
    assert _rel(G, (X.float() @ W.float().t()) * gp.float()) < 4e-3
    # N % 8 == 4: the last 8-column group holds 4 valid columns
    Nr = 132
    Cr = torch.empty(M, Nr, device=dev, dtype=torch.bfloat16)
    gr = torch.empty(M, Nr, device=dev, dtype=torch.bfloat16)
    Wr = (torch.randn(Nr, Kk, device=dev) * 0.1).bfloat16()
    br = torch.randn(Nr, device=dev)
    refr = X.float() @ Wr.float().t() + br
    with pytest.raises(RuntimeError):   # ldc % 8 != 0 is rejected for the vectorised epilogue
        K.gemm(X, Wr, Cr, M, Nr, Kk, epi=N.EPI_BF16, bias=br)
    Cp = torch.empty(M, 136, device=dev, dtype=torch.bfloat16)
    K.gemm(X, Wr, Cp, M, Nr, Kk, epi=N.EPI_BF16, bias=br, ldc=136)
    assert _rel(Cp[:, :Nr], refr) < 4e-3
    C32r = torch.empty(M, 136, device=dev)
    K.gemm(X, Wr, C32r, M, Nr, Kk, epi=N.EPI_F32, bias=br, ldc=136)
    assert _rel(C32r[:, :Nr], refr) < 1e-5
    # residual f32
    R = torch.randn(M, Nn, device=dev)
    C32 = torch.empty(M, Nn, device=dev)
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_F32, bias=b, resid=R, ldr=Nn)
    assert _rel(C32, ref + R) < 1e-5
    # dropout + residual: kept fraction ~ 0.9, kept values scaled by 1/0.9
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=Nn, drop_p=0.1, seed=123)
    acc = X.float() @ W.float().t()
    keep = (C32 - R).abs() > 1e-6
    assert 0.87 < keep.float().mean().item() < 0.93
    assert _rel((C32 - R)[keep], (acc / 0.9)[keep]) < 1e-5
    # the backward cast regenerates the same mask
    gb = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.dropout_bwd_cast(torch.ones(M, Nn, device=dev), gb, 0.1, 123, M, Nn)
    agree = ((gb.float() != 0) == keep) | (acc.abs() < 1e-4)
    assert agree.all()


@pytest.mark.parametrize('M,Nn,Kk', [(32768, 512, 256), (1024, 512, 512), (1000, 520, 2048), (48, 512, 256)])
def test_gemm_dropout_resid_bf16_copy(M, Nn, Kk):
    # DROPOUT_RESID with aux: the epilogue's bf16 copy of the f32 output (the last decoder layer -> the vocab head's
    # input) equals the round-to-nearest bf16 of C exactly, in every kernel (256x256 persistent, LDS-DMA, skinny)
    torch.manual_seed(M + Kk)
    X = torch.randn(M, Kk, device=dev).bfloat16()
    W = (torch.randn(Nn, Kk, device=dev) * 0.1).bfloat16()
    R = torch.randn(M, Nn, device=dev)
    C32 = torch.empty(M, Nn, device=dev)
    Cb = torch.full((M, Nn), float('nan'), device=dev, dtype=torch.bfloat16)
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=Nn, drop_p=0.1, seed=9, aux=Cb, ldaux=Nn)
    C0 = torch.empty(M, Nn, device=dev)
    K.gemm(X, W, C0, M, Nn, Kk, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=Nn, drop_p=0.1, seed=9)
    torch.cuda.synchronize()
    assert torch.equal(C32, C0)                       # the f32 output is unchanged by the copy
    assert torch.equal(Cb, C32.bfloat16())
    with pytest.raises(RuntimeError):                 # ldaux % 8 != 0 is rejected
        K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=Nn, aux=Cb, ldaux=Nn - 4)


@pytest.mark.parametrize('M,Nn,Kk', [(64, 512, 2048), (37, 520, 72), (1, 2048, 512), (64, 512, 64)])
def test_gemm_skinny_epilogues(M, Nn, Kk):
    # M <= 64: the K-split skinny kernel (one row per sequence: encoder bottleneck, q(z|x), z projections)
    torch.manual_seed(M + Nn + Kk)
    Ai = torch.randint(-2, 3, (M, Kk), device=dev).float()
    Bi = torch.randint(-2, 3, (Nn, Kk), device=dev).float()
    C32 = torch.empty(M, Nn, device=dev)
    K.gemm(Ai.bfloat16(), Bi.bfloat16(), C32, M, Nn, Kk, epi=N.EPI_F32)
    torch.cuda.synchronize()
    assert torch.equal(C32, Ai @ Bi.t())
    X = torch.randn(M, Kk, device=dev).bfloat16()
    W = (torch.randn(Nn, Kk, device=dev) * 0.1).bfloat16()
    b = torch.randn(Nn, device=dev)
    acc = X.float() @ W.float().t()
    ref = acc + b
    C = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_BF16, bias=b)
    assert _rel(C, ref) < 4e-3
    gp = torch.empty_like(C)
    K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_GELU, bias=b, aux=gp, ldaux=Nn)
    r = ref.clone().requires_grad_()
    F.gelu(r).backward(torch.ones_like(r))
    assert _rel(C, F.gelu(ref)) < 4e-3 and _rel(gp, r.grad) < 4e-3
    G = torch.empty_like(C)
    K.gemm(X, W, G, M, Nn, Kk, epi=N.EPI_GELU_BWD, aux=gp, ldaux=Nn)
    assert _rel(G, acc * gp.float()) < 4e-3
    R = torch.randn(M, Nn, device=dev)
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_F32, bias=b, resid=R, ldr=Nn)
    assert _rel(C32, ref + R) < 1e-5
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=Nn, drop_p=0.25, seed=7)
    gb = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.dropout_bwd_cast(torch.ones(M, Nn, device=dev), gb, 0.25, 7, M, Nn)
    keep = gb.float() != 0
    assert torch.allclose((C32 - R)[keep], (acc / 0.75)[keep], rtol=1e-4, atol=1e-4)
    assert torch.allclose((C32 - R)[~keep], torch.zeros_like(R)[~keep], atol=1e-6)
    # strided f32 output rows (the z splice writes row 0 of every sequence: ldc = L * d)
    Cs = torch.zeros(M, 2 * Nn, device=dev)
    K.gemm(X, W, Cs, M, Nn, Kk, epi=N.EPI_F32, bias=b, ldc=2 * Nn)
    assert _rel(Cs[:, :Nn], ref) < 1e-5 and torch.all(Cs[:, Nn:] == 0)


@pytest.mark.parametrize('M,Nn,Kk', [(8200, 2056, 520), (8192, 2048, 512)])
def test_gemm_many_tiles_epilogues(M, Nn, Kk):
    # >= 512 tiles of 256 x 128: the shapes gemm_ov takes when enabled (SVAE_GEMM_OV=1; ragged M, N, K in the first)
    torch.manual_seed(M + Kk)
    Ai = torch.randint(-2, 3, (M, Kk), device=dev).float()
    Bi = torch.randint(-2, 3, (Nn, Kk), device=dev).float()
    C32 = torch.empty(M, Nn, device=dev)
    K.gemm(Ai.bfloat16(), Bi.bfloat16(), C32, M, Nn, Kk, epi=N.EPI_F32)
    torch.cuda.synchronize()
    assert torch.equal(C32, Ai @ Bi.t())
    X = torch.randn(M, Kk, device=dev).bfloat16()
    W = (torch.randn(Nn, Kk, device=dev) * 0.1).bfloat16()
    b = torch.randn(Nn, device=dev)
    acc = X.float() @ W.float().t()
    ref = acc + b
    C = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_BF16, bias=b)
    assert _rel(C, ref) < 4e-3
    gp = torch.empty_like(C)
    K.gemm(X, W, C, M, Nn, Kk, epi=N.EPI_GELU, bias=b, aux=gp, ldaux=Nn)
    r = ref.clone().requires_grad_()
    F.gelu(r).backward(torch.ones_like(r))
    assert _rel(C, F.gelu(ref)) < 4e-3 and _rel(gp, r.grad) < 4e-3
    G = torch.empty_like(C)
    K.gemm(X, W, G, M, Nn, Kk, epi=N.EPI_GELU_BWD, aux=gp, ldaux=Nn)
    assert _rel(G, acc * gp.float()) < 4e-3
    R = torch.randn(M, Nn, device=dev)
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_F32, bias=b, resid=R, ldr=Nn)
    assert _rel(C32, ref + R) < 1e-5
    K.gemm(X, W, C32, M, Nn, Kk, epi=N.EPI_DROPOUT_RESID, resid=R, ldr=Nn, drop_p=0.1, seed=123)
    keep = (C32 - R).abs() > 1e-6
    assert 0.87 < keep.float().mean().item() < 0.93
    assert _rel((C32 - R)[keep], (acc / 0.9)[keep]) < 1e-5
    gb = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.dropout_bwd_cast(torch.ones(M, Nn, device=dev), gb, 0.1, 123, M, Nn)
    assert (((gb.float() != 0) == keep) | (acc.abs() < 1e-4)).all()


@pytest.mark.parametrize('B,L,d', [(2, 96, 256), (16, 512, 512), (24, 512, 512)])
def test_gemm_rotary_matches_reference_rotation(B, L, d):
    torch.manual_seed(1)
    X = torch.randn(B * L, d, device=dev).bfloat16()
    W = (torch.randn(3 * d, d, device=dev) * 0.05).bfloat16()
    b = torch.randn(3 * d, device=dev) * 0.1
    rot = rotary_table(L, d).to(dev)
    C = torch.empty(B * L, 3 * d, device=dev, dtype=torch.bfloat16)
    K.gemm(X, W, C, B * L, 3 * d, d, epi=N.EPI_ROTARY_BF16, bias=b, rot=rot, rot_cols=2 * d, rot_d=d, rot_seq=L)
    y = (X.float() @ W.float().t() + b).view(B, L, 3 * d).cpu()
    ref = torch.cat([oracle.rotary(y[..., :d]), oracle.rotary(y[..., d:2 * d]), y[..., 2 * d:]], -1)
    assert _rel(C.view(B, L, 3 * d).cpu(), ref) < 4e-3


@pytest.mark.parametrize('T', [256, 512])
def test_ce_stats_epilogue_and_finalize(T):
    torch.manual_seed(2)
    d, V, L = 128, 32768, 128
    X = torch.randn(T, d, device=dev).bfloat16()
    W = (torch.randn(V, d, device=dev) * 0.1).bfloat16()
    b = torch.randn(V, device=dev) * 0.1
    labels = torch.randint(0, V, (T,), device=dev, dtype=torch.int32)
    labels[::7] = 0
    logits = torch.empty(T, V, device=dev, dtype=torch.bfloat16)
    ntile = V // 128
    part = torch.empty(T, ntile, 2, device=dev)
    ll = torch.zeros(T, device=dev)
    K.gemm(X, W, logits, T, V, d, epi=N.EPI_CE_STATS, bias=b, aux=part, labels=labels, label_logit=ll)
    ref = X.float() @ W.float().t() + b
    lse, rl, cw, nll = (torch.empty(T, device=dev), torch.empty(T, device=dev), torch.empty(8, device=dev),
                        torch.empty(1, device=dev))
    K.ce_finalize(part, ntile, ll, labels, T, L, 1, L, lse, rl, cw, nll)
    assert _rel(lse, ref.logsumexp(-1)) < 1e-6
    nll_ref = F.cross_entropy(ref, labels.long(), ignore_index=0)
    assert abs(nll.item() - nll_ref.item()) / nll_ref.item() < 1e-5
    gs = torch.ones(1, device=dev)
    db = torch.zeros(V, device=dev)
    K.ce_grad(logits, V, lse, cw, labels, gs, T, V, L, 1, L, dbias=db)
    r = ref.clone().requires_grad_()
    F.cross_entropy(r, labels.long(), ignore_index=0).backward()
    assert _rel(logits, r.grad) < 1e-2
    assert _rel(db, r.grad.sum(0)) < 1e-2


@pytest.mark.parametrize('D,xdt', [(128, torch.float32), (384, torch.float32), (512, torch.bfloat16), (768, torch.float32)])
def test_layernorm(D, xdt):
    torch.manual_seed(D)
    rows = 333
    x = (torch.randn(rows, D, device=dev) * 2 + 0.5).to(xdt)
    w = torch.randn(D, device=dev) * 0.1 + 1
    bb = torch.randn(D, device=dev) * 0.1
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_fwd(x, w, bb, y, mean, rstd, rows, D)
    xr = x.float().requires_grad_()
    wr, br = w.clone().requires_grad_(), bb.clone().requires_grad_()
    ref = F.layer_norm(xr, (D,), wr, br, 1e-5)
    assert _rel(y, ref) < 4e-3
    dy = torch.randn(rows, D, device=dev).bfloat16()
    ref.backward(dy.float())
    dres = torch.randn(rows, D, device=dev)
    dx = torch.empty(rows, D, device=dev)
    dxb = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    wg = torch.zeros(2 * D, device=dev)
    part = torch.empty(1024 * 2 * D, device=dev)
    K.layernorm_bwd(dy, x, w, mean, rstd, dres, dx, dxb, wg, rows, D, part)
    assert _rel(dx, xr.grad + dres) < 1e-4
    assert _rel(dxb, xr.grad + dres) < 4e-3
    assert _rel(wg[:D], wr.grad) < 1e-4 and _rel(wg[D:], br.grad) < 1e-4


@pytest.mark.parametrize('p', [0.0, 0.1, 0.5])
def test_layernorm_bwd_fused_dropout_cast(p):
    # the bf16 copy with the next layer's dropout backward + position-0 zeroing equals the unfused sequence
    # (layernorm_bwd, then dropout_bwd_cast of dx with rows % L == 0 zeroed) bit for bit; dx itself is unchanged
    D, L, rows = 512, 64, 64 * 7
    torch.manual_seed(11)
    x = torch.randn(rows, D, device=dev) * 2 + 0.5
    w = torch.randn(D, device=dev) * 0.1 + 1
    bb = torch.randn(D, device=dev) * 0.1
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_fwd(x, w, bb, y, mean, rstd, rows, D)
    dy = torch.randn(rows, D, device=dev).bfloat16()
    dres = torch.randn(rows, D, device=dev)
    part = torch.empty(1024 * 2 * D, device=dev)
    seed = 0x9E3779B97F4A7C15
    dx0, wg0 = torch.empty(rows, D, device=dev), torch.zeros(2 * D, device=dev)
    K.layernorm_bwd(dy, x, w, mean, rstd, dres, dx0, None, wg0, rows, D, part)
    ref = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    dxz = dx0.clone()
    dxz[::L] = 0
    K.dropout_bwd_cast(dxz, ref, p, seed, rows, D)
    dx1, wg1 = torch.empty(rows, D, device=dev), torch.zeros(2 * D, device=dev)
    got = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    K.layernorm_bwd(dy, x, w, mean, rstd, dres, dx1, got, wg1, rows, D, part, bf_drop=(p, seed, L))
    torch.cuda.synchronize()
    assert torch.equal(dx1, dx0) and torch.equal(got, ref)
    assert torch.allclose(wg1, wg0, rtol=1e-6, atol=1e-6)
    if p > 0:
        assert (got.float() == 0).float().mean().item() > p * 0.8
    # + the z splice: rows r % L == 0 move to zrow / zrow_bf and are zeroed in dx (extract_rows + cast_bf16)
    zr, zb = torch.full((rows // L, D), 7.0, device=dev), torch.zeros(rows // L, D, device=dev, dtype=torch.bfloat16)
    dx2, got2 = torch.empty(rows, D, device=dev), torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    K.layernorm_bwd(dy, x, w, mean, rstd, dres, dx2, got2, torch.zeros(2 * D, device=dev), rows, D, part,
                    bf_drop=(p, seed, L), zsplice=(L, zr, zb))
    torch.cuda.synchronize()
    assert torch.equal(zr, dx0[::L]) and torch.equal(zb, dx0[::L].bfloat16())
    assert torch.equal(dx2, dxz) and torch.equal(got2, ref)


@pytest.mark.parametrize('D,rows,xdt', [(512, 64 * 9, torch.float32), (768, 300, torch.float32), (256, 77, torch.bfloat16)])
def test_layernorm_bwd_gelu_fused(D, rows, xdt):
    # the head LayerNorm's backward fused with the GELU backward before it: bf16(LN'(dy) * gp) equals layernorm_bwd
    # then gelu_bwd bit for bit, and the affine gradients are the same
    torch.manual_seed(D + rows)
    x = (torch.randn(rows, D, device=dev) * 2 + 0.5).to(xdt)
    w = torch.randn(D, device=dev) * 0.1 + 1
    bb = torch.randn(D, device=dev) * 0.1
    y = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_fwd(x, w, bb, y, mean, rstd, rows, D)
    dy = torch.randn(rows, D, device=dev).bfloat16()
    gp = torch.rand(rows, D, device=dev).bfloat16() * 1.2 - 0.1
    part = torch.empty(1024 * 2 * D, device=dev)
    dx0, wg0 = torch.empty(rows, D, device=dev), torch.zeros(2 * D, device=dev)
    K.layernorm_bwd(dy, x, w, mean, rstd, None, dx0, None, wg0, rows, D, part)
    ref = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    K.gelu_bwd(dx0, gp, ref, rows * D)
    got, wg1 = torch.full((rows, D), float('nan'), device=dev, dtype=torch.bfloat16), torch.zeros(2 * D, device=dev)
    K.layernorm_bwd_gelu(dy, x, w, mean, rstd, gp, got, wg1, rows, D, part)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert torch.equal(wg1, wg0)


@pytest.mark.parametrize('M,Nn,Kk,p', [(32768, 512, 512, 0.1), (1024, 512, 256, 0.25), (1000, 520, 2048, 0.0),
                                       (48, 512, 256, 0.1)])
def test_gemm_f32_dropout_bf16_copy(M, Nn, Kk, p):
    # EPI_F32 with aux: C unchanged, aux = what dropout_bwd_cast makes of C (the head's d x -> the top decoder layer's
    # dropout-masked FFN-output gradient), bit for bit, in the 256x256 persistent, LDS-DMA and skinny kernels
    torch.manual_seed(M + Kk)
    X = torch.randn(M, Kk, device=dev).bfloat16()
    W = (torch.randn(Nn, Kk, device=dev) * 0.1).bfloat16()
    b = torch.randn(Nn, device=dev)
    seed = 0x243F6A8885A308D3
    C0 = torch.empty(M, Nn, device=dev)
    K.gemm(X, W, C0, M, Nn, Kk, epi=N.EPI_F32, bias=b)
    C1 = torch.empty(M, Nn, device=dev)
    got = torch.full((M, Nn), float('nan'), device=dev, dtype=torch.bfloat16)
    K.gemm(X, W, C1, M, Nn, Kk, epi=N.EPI_F32, bias=b, aux=got, ldaux=Nn, drop_p=p, seed=seed)
    ref = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.dropout_bwd_cast(C0, ref, p, seed, M, Nn)
    torch.cuda.synchronize()
    assert torch.equal(C1, C0)
    assert torch.equal(got, ref)


@pytest.mark.parametrize('B,L,mode', [(64, 512, 'bool'), (3, 37, 'ids'), (5, 1, 'none'), (300, 64, 'bool')])
def test_prep_tokens(B, L, mode):
    # the step's token inputs in one launch equal the torch op sequence it replaces
    torch.manual_seed(B + L)
    ids = torch.randint(0, 5, (B, L), device=dev, dtype=torch.int64) * 7919
    pad = {'bool': ids.eq(0), 'ids': True, 'none': None}[mode]
    ntok = torch.randint(1, L + 1, (B,), device=dev, dtype=torch.int64)
    ids32 = torch.full((B, L), -5, device=dev, dtype=torch.int32)
    labels = torch.full((B, L), -5, device=dev, dtype=torch.int32)
    padm = torch.full((B, L), 9, device=dev, dtype=torch.uint8) if pad is not None else None
    nt = torch.full((B,), -1, device=dev, dtype=torch.int64)
    K.prep_tokens(ids, pad, B, L, ids32, labels, padm, ntok, nt)
    torch.cuda.synchronize()
    assert torch.equal(ids32, ids.to(torch.int32))
    ref = torch.zeros(B, L, device=dev, dtype=torch.int32)
    ref[:, :-1] = ids[:, 1:].to(torch.int32)
    assert torch.equal(labels, ref)
    if padm is not None:
        assert torch.equal(padm, ids.eq(0).to(torch.uint8))
    assert torch.equal(nt, ntok)


@pytest.mark.parametrize('n,B,d,Z', [(6, 64, 512, 64), (3, 5, 200, 70), (12, 130, 768, 128)])
def test_zproj_fwd_multi(n, B, d, Z):
    # n z projections in one launch: z W_i^T + b_i against torch fp32 on the same bf16 operands
    torch.manual_seed(n + B + d + 1)
    z = torch.randn(B, Z, device=dev).bfloat16()
    Ws = [(torch.randn(d, Z, device=dev) * 0.1).bfloat16() for _ in range(n)]
    bs = [torch.randn(d, device=dev) for _ in range(n)]
    outs = [torch.full((B, d), float('nan'), device=dev) for _ in range(n)]
    K.zproj_fwd_multi([(Ws[i], bs[i], outs[i]) for i in range(n)], z, B, d, Z)
    torch.cuda.synchronize()
    for i in range(n):
        ref = z.float() @ Ws[i].float().t() + bs[i]
        assert torch.allclose(outs[i], ref, rtol=1e-5, atol=1e-5)


@pytest.mark.parametrize('rows,L,D', [(64 * 512, 512, 512), (3 * 40, 40, 768), (7 * 16, 16, 256)])
def test_layernorm_fwd_zsplice(rows, L, D):
    # the layer's first LayerNorm with the z splice equals writing the z rows into x, then the plain LayerNorm
    torch.manual_seed(rows + D)
    x = torch.randn(rows, D, device=dev) * 2 + 0.3
    zr = torch.randn(rows // L, D, device=dev)
    w = torch.randn(D, device=dev) * 0.1 + 1
    bb = torch.randn(D, device=dev) * 0.1
    x_ref = x.clone()
    x_ref[::L] = zr
    y0 = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    m0, r0 = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_fwd(x_ref, w, bb, y0, m0, r0, rows, D)
    y1 = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    m1, r1 = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_fwd_z(x, zr, L, w, bb, y1, m1, r1, rows, D)
    torch.cuda.synchronize()
    assert torch.equal(x, x_ref)
    assert torch.equal(y1, y0) and torch.equal(m1, m0) and torch.equal(r1, r0)


@pytest.mark.parametrize('n,rows,D', [(4, 4100, 768), (3, 333, 512), (1, 77, 768), (2, 300, 96), (4, 65, 1024)])
def test_layernorm_multi_matches_per_layer(n, rows, D):
    # the encoder middle layers' context LayerNorms batched (one input, n affines): the forward equals n layernorm_fwd
    # calls bit for bit; the backward's dx equals dres + the n layernorm_bwd contributions and each affine gradient
    # equals its own pass's (up to f32 summation order: LN' summed before the row reductions)
    torch.manual_seed(n + rows + D)
    x = torch.randn(rows, D, device=dev) * 2 + 0.5
    ws = [torch.randn(D, device=dev) * 0.1 + 1 for _ in range(n)]
    bs = [torch.randn(D, device=dev) * 0.1 for _ in range(n)]
    ys0 = [torch.empty(rows, D, device=dev, dtype=torch.bfloat16) for _ in range(n)]
    m0, r0 = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    for j in range(n):
        K.layernorm_fwd(x, ws[j], bs[j], ys0[j], m0, r0, rows, D)
    ys1 = [torch.full((rows, D), float('nan'), device=dev, dtype=torch.bfloat16) for _ in range(n)]
    m1, r1 = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.layernorm_fwd_multi(x, ws, bs, ys1, m1, r1, rows, D)
    torch.cuda.synchronize()
    assert torch.equal(m1, m0) and torch.equal(r1, r0)
    assert all(torch.equal(a, b) for a, b in zip(ys0, ys1))
    dys = [torch.randn(rows, D, device=dev).bfloat16() for _ in range(n)]
    dres = torch.randn(rows, D, device=dev)
    part = torch.empty(N.LN_MULTI_MAX * 1024 * 2 * D, device=dev)
    dx0, wg0 = dres.clone(), [torch.zeros(2 * D, device=dev) for _ in range(n)]
    for j in range(n):
        K.layernorm_bwd(dys[j], x, ws[j], m0, r0, dx0, dx0, None, wg0[j], rows, D, part)
    dx1, wg1 = dres.clone(), [torch.zeros(2 * D, device=dev) for _ in range(n)]
    K.layernorm_bwd_multi(dys, x, ws, m1, r1, dx1, dx1, wg1, rows, D, part)
    torch.cuda.synchronize()
    assert _rel(dx1, dx0) < 1e-6
    for j in range(n):
        assert _rel(wg1[j], wg0[j]) < 1e-6


@pytest.mark.parametrize('n,B,d,Z', [(6, 64, 512, 64), (3, 5, 200, 70), (12, 130, 768, 128)])
def test_zproj_bwd_multi_matches_sequential(n, B, d, Z):
    # n z-projection backwards in one launch equal n svae_zproj_bwd calls in list order, bit for bit (dW, db, dz)
    torch.manual_seed(n + B + d)
    z = torch.randn(B, Z, device=dev).bfloat16()
    dz0 = torch.randn(B, Z, device=dev)
    gs = [torch.randn(B, d, device=dev) for _ in range(n)]
    Ws = [(torch.randn(d, Z, device=dev) * 0.1).bfloat16() for _ in range(n)]
    dW0 = [torch.randn(d, Z, device=dev) for _ in range(n)]
    db0 = [torch.randn(d, device=dev) for _ in range(n)]
    dz_a, dW_a, db_a = dz0.clone(), [t.clone() for t in dW0], [t.clone() for t in db0]
    for i in range(n):
        K.zproj_bwd(gs[i], z, Ws[i], dW_a[i], db_a[i], dz_a, B, d, Z)
    dz_b, dW_b, db_b = dz0.clone(), [t.clone() for t in dW0], [t.clone() for t in db0]
    K.zproj_bwd_multi([(gs[i], Ws[i], dW_b[i], db_b[i]) for i in range(n)], z, dz_b, B, d, Z)
    torch.cuda.synchronize()
    assert torch.equal(dz_a, dz_b)
    for i in range(n):
        assert torch.equal(dW_a[i], dW_b[i]) and torch.equal(db_a[i], db_b[i])


@pytest.mark.parametrize('kw', [0.3, 0.7123, 1.0])
def test_step_scalars(kw):
    # loss = nll + kw * kl and gs = (gloss, gloss * kw): bit-equal to the torch expressions they replace
    nll = torch.tensor([7.123456], device=dev)
    kl = torch.tensor([1.98765], device=dev)
    gl = torch.tensor([0.3333333], device=dev)
    loss, gs = torch.empty(1, device=dev), torch.empty(2, device=dev)
    K.step_scalars(kw, nll=nll, kl=kl, loss=loss)
    K.step_scalars(kw, gloss=gl, gs=gs)
    torch.cuda.synchronize()
    assert torch.equal(loss[0], nll[0] + kw * kl[0])
    assert torch.equal(gs, torch.cat([gl, gl * kw]))


@pytest.mark.parametrize('B,d,Z', [(64, 512, 64), (3, 200, 70), (130, 768, 128)])
def test_zproj_bwd(B, d, Z):
    # z_projections backward in one launch: dW += g^T z, db += sum_b g, dz += g W (f32 accumulation; z, W bf16)
    torch.manual_seed(B + d + Z)
    g = torch.randn(B, d, device=dev)
    z = torch.randn(B, Z, device=dev).bfloat16()
    W = (torch.randn(d, Z, device=dev) * 0.1).bfloat16()
    dW, db, dz = torch.randn(d, Z, device=dev), torch.randn(d, device=dev), torch.randn(B, Z, device=dev)
    rW = dW + g.double().t().mm(z.double()).float()
    rb = db + g.double().sum(0).float()
    rz = dz + g.double().mm(W.double()).float()
    K.zproj_bwd(g, z, W, dW, db, dz, B, d, Z)
    torch.cuda.synchronize()
    assert _rel(dW, rW) < 1e-6 and _rel(db, rb) < 1e-6 and _rel(dz, rz) < 1e-6


@pytest.mark.parametrize('rows,cols,ld,dt', [(1024, 1024, 1024, torch.float32), (1000, 512, 520, torch.float32),
                                            (37, 1024, 1024, torch.float32), (5, 8, 8, torch.float32),
                                            (32768, 512, 512, torch.bfloat16), (4093, 2048, 2048, torch.bfloat16)])
def test_colsum(rows, cols, ld, dt):
    # column sums (bias / LayerNorm-affine gradients): unrolled row groups + ragged tails, accumulate into out
    torch.manual_seed(rows + cols)
    x = torch.randn(rows, ld, device=dev).to(dt)
    out = torch.randn(cols, device=dev)
    ref = out + x[:, :cols].double().sum(0).float()
    K.colsum(x, rows, cols, ld, out, accumulate=True)
    torch.cuda.synchronize()
    assert _rel(out, ref) < 1e-5


def _attn_ref(q, k, v, pad, causal, scale):
    s = q @ k.transpose(-1, -2) * scale
    mask = None
    if pad is not None:
        mask = pad[:, None, None, :].bool()
    if causal:
        cm = torch.ones(q.shape[-2], k.shape[-2], device=q.device, dtype=torch.bool).triu(1)
        mask = cm if mask is None else mask | cm
    if mask is not None:
        s = s - mask * 1e7
    return s.softmax(-1) @ v


@pytest.mark.parametrize('B,H,Lq,Lk,hd,causal,padded,learned', [
    (2, 4, 128, 128, 64, True, True, False),
    (2, 2, 192, 192, 64, True, False, False),
    (2, 3, 64, 200, 64, False, True, True),
    (3, 2, 1, 64, 64, False, False, True),
    (2, 2, 96, 96, 96, True, True, False),
    (1, 2, 130, 130, 32, True, False, False),
    (2, 8, 64, 64, 16, False, False, False),
    (2, 2, 512, 512, 64, True, True, False),
    (1, 2, 300, 520, 64, False, True, False),
    (1, 2, 1024, 1024, 96, True, True, False),     # C4 decoder head dim: 4 key blocks of 256, ragged padding
    (2, 2, 600, 600, 96, True, False, False),      # hd 96, last key block partial (600 = 2 x 256 + 88)
    (2, 4, 64, 520, 64, False, True, True),        # learned queries over 3 key blocks (the encoder's first layer)
    (1, 2, 1536, 1536, 64, True, False, False),    # 3 dQ planes of two 256-key sub-blocks each
    (1, 2, 256, 1300, 96, False, True, False),     # non-causal hd 96: 6 sub-blocks, the last partial, 3 planes
    # few queries over many keys: the split-KV forward (key slices + combine), learned queries / padding / hd 96
    (2, 2, 64, 5000, 64, False, True, True),
    (1, 2, 100, 3000, 64, False, False, False),
    (1, 2, 64, 4100, 96, False, True, False),
])
def test_attention_fwd_bwd(B, H, Lq, Lk, hd, causal, padded, learned):
    torch.manual_seed(Lq * 7 + hd)
    d = H * hd
    q = torch.randn(1 if learned else B, Lq, d, device=dev).bfloat16()
    k = torch.randn(B, Lk, d, device=dev).bfloat16()
    v = torch.randn(B, Lk, d, device=dev).bfloat16()
    pad = None
    if padded:
        pad = torch.zeros(B, Lk, device=dev, dtype=torch.uint8)
        for b in range(B):
            pad[b, Lk - 1 - 17 * b - 5:] = 1
    o = torch.empty(B, Lq, d, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, Lq, device=dev)
    scale = hd ** -0.5
    common = dict(B=B, H=H, Lq=Lq, Lk=Lk, hd=hd, sq=d, bq=0 if learned else Lq * d, sk=d, sv=d, bk=Lk * d,
                  bv=Lk * d, so=d, bo=Lq * d, key_pad=pad, causal=causal)
    K.attention(q, k, v, o, lse, **common)

    def heads(t):
        return t.float().view(t.shape[0], t.shape[1], H, hd).transpose(1, 2)

    qr = heads(q).expand(B, -1, -1, -1).clone().requires_grad_()
    kr, vr = heads(k).requires_grad_(), heads(v).requires_grad_()
    ref = _attn_ref(qr, kr, vr, pad, causal, scale)
    ref_o = ref.transpose(1, 2).reshape(B, Lq, d)
    assert _rel(o, ref_o) < 1e-2
    with torch.no_grad():   # lse (the backward's row constant; the split-KV forward combines it over key slices)
        sc = qr @ kr.transpose(-1, -2) * scale
        if pad is not None:
            sc = sc - pad[:, None, None, :].float() * 1e7
        if causal:
            sc = sc - torch.ones(Lq, Lk, device=dev).triu(1) * 1e7
        assert (lse - torch.logsumexp(sc, -1)).abs().max().item() < 1e-4
    do = torch.randn(B, Lq, d, device=dev).bfloat16()
    ref_o.backward(do.float())
    dq = torch.full((B, Lq, d), 7.0, device=dev)    # written, not accumulated
    dk = torch.empty(B, Lk, d, device=dev, dtype=torch.bfloat16)
    dv = torch.empty_like(dk)
    delta = torch.empty(B, H, Lq, device=dev)
    K.attention(q, k, v, o, lse, backward=True, dout=do, sdo=d, bdo=Lq * d, delta=delta, dq=dq, bdq=Lq * d,
                dk=dk, dv=dv, sdk=d, sdv=d, bdk=Lk * d, bdv=Lk * d, **common)

    def unheads(t):
        return t.transpose(1, 2).reshape(t.shape[0], t.shape[2], d)

    assert _rel(dq, unheads(qr.grad)) < 2e-2
    assert _rel(dk, unheads(kr.grad)) < 2e-2
    assert _rel(dv, unheads(vr.grad)) < 2e-2


@pytest.mark.parametrize('hd,L,causal', [(64, 1024, True), (96, 1024, True), (128, 512, True), (64, 520, False)])
def test_attention_bwd_row_constant_slots_repeatable(hd, L, causal):
    """The backward kernels take each query tile's lse and delta rows through a per-wave LDS slot filled by LDS-DMA
    (the protocol whose k-weighted GEMM form once read stale slots). Here the query tiles' lse and delta
    differ by large factors (Q and dO scaled per 64-query tile), so a slot read one tile stale would move dQ / dK / dV
    far past the tolerance; 20 repeated backwards must also be bit-identical (the kernels are deterministic: no float
    atomics), which catches an intermittent stale read even where its effect is small."""
    torch.manual_seed(hd + L)
    B, H = 4, 3
    d = H * hd
    nt = (L + 63) // 64
    f = torch.tensor([0.25, 2.0, 0.5, 3.0, 1.0, 0.35, 2.5, 0.7], device=dev).repeat(nt)[:nt].repeat_interleave(64)[:L]
    q = (torch.randn(B, L, d, device=dev) * f[None, :, None]).bfloat16()
    k = torch.randn(B, L, d, device=dev).bfloat16()
    v = torch.randn(B, L, d, device=dev).bfloat16()
    do = (torch.randn(B, L, d, device=dev) * f.flip(0)[None, :, None] * 4).bfloat16()
    pad = None
    if not causal:
        pad = torch.zeros(B, L, device=dev, dtype=torch.uint8)
        pad[:, L - 37:] = 1
    o = torch.empty(B, L, d, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    o32 = torch.empty(B, L, d, device=dev)
    common = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=d, bq=L * d, sk=d, sv=d, bk=L * d, bv=L * d, so=d, bo=L * d,
                  key_pad=pad, causal=causal)
    K.attention(q, k, v, o, lse, o32=o32, so32=d, bo32=L * d, **common)
    runs = []
    for _ in range(20):
        dq = torch.empty(B, L, d, device=dev)
        dk = torch.empty(B, L, d, device=dev, dtype=torch.bfloat16)
        dv = torch.empty_like(dk)
        delta = torch.empty(B, H, L, device=dev)
        K.attention(q, k, v, o, lse, backward=True, dout=do, sdo=d, bdo=L * d, delta=delta, dq=dq, bdq=L * d,
                    dk=dk, dv=dv, sdk=d, sdv=d, bdk=L * d, bdv=L * d, o32=o32, so32=d, bo32=L * d, **common)
        runs.append((dq, dk, dv))
    torch.cuda.synchronize()
    for i, r in enumerate(runs[1:], 1):
        for name, a, b in zip(('dq', 'dk', 'dv'), runs[0], r):
            assert torch.equal(a, b), (i, name, (a.float() - b.float()).abs().max().item())

    def heads(t):
        return t.float().view(B, L, H, hd).transpose(1, 2)

    qr, kr, vr = (heads(t).requires_grad_() for t in (q, k, v))
    ref = _attn_ref(qr, kr, vr, pad, causal, hd ** -0.5).transpose(1, 2).reshape(B, L, d)
    ref.backward(do.float())

    def unheads(t):
        return t.transpose(1, 2).reshape(B, L, d)

    dq, dk, dv = runs[0]
    assert _rel(dq, unheads(qr.grad)) < 2e-2
    assert _rel(dk, unheads(kr.grad)) < 2e-2
    assert _rel(dv, unheads(vr.grad)) < 2e-2


@pytest.mark.parametrize('hd,L', [(64, 512), (96, 1024), (32, 130), (64, 1100), (64, 300)])
def test_attention_o_lo_matches_o32(hd, L):
    """The forward's bf16 residual o_lo = O - bf16(O) carries the f32 O to ~16 bits: delta from (O, o_lo) -- the
    separate pass, or at hd <= 64 computed inside the 8-wave backward from LDS-DMA'd O / o_lo rows -- gives the
    backward of the f32 copy o32 to ~1e-5."""
    torch.manual_seed(hd * 3 + L)
    B, H = 2, 3
    d = H * hd
    qkv = torch.randn(B * L, 3 * d, device=dev).bfloat16()
    common = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=3 * d, bq=L * 3 * d, sk=3 * d, sv=3 * d, bk=L * 3 * d,
                  bv=L * 3 * d, so=d, bo=L * d, causal=True)
    o, o2 = (torch.empty(B * L, d, device=dev, dtype=torch.bfloat16) for _ in range(2))
    lse, lse2 = torch.empty(B, H, L, device=dev), torch.empty(B, H, L, device=dev)
    o32 = torch.empty(B * L, d, device=dev)
    olo = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, o32=o32, so32=d, bo32=L * d, **common)
    K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o2, lse2, o_lo=olo, so_lo=d, bo_lo=L * d, **common)
    assert torch.equal(o, o2) and torch.equal(lse, lse2)
    assert torch.equal(o.float(), o32.bfloat16().float())                 # O is bf16(o32)
    assert (o.float() + olo.float() - o32).abs().max() <= o32.abs().max() * 2.0 ** -16
    do = torch.randn(B * L, d, device=dev).bfloat16()
    outs = []
    for extra in (dict(o32=o32, so32=d, bo32=L * d), dict(o_lo=olo, so_lo=d, bo_lo=L * d)):
        delta = torch.empty(B, H, L, device=dev)
        g = torch.empty(B * L, 3 * d, device=dev, dtype=torch.bfloat16)
        K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, backward=True, dout=do, sdo=d, bdo=L * d, delta=delta,
                    dq_bf=g, ldq_bf=3 * d, dk=g[:, d:], dv=g[:, 2 * d:], sdk=3 * d, sdv=3 * d, bdk=L * 3 * d,
                    bdv=L * 3 * d, **extra, **common)
        outs.append((delta.clone(), g.float()))
    (d32, g32), (dlo, glo) = outs
    assert _rel(dlo, d32) < 1e-5
    assert _rel(glo, g32) < 1e-3      # bf16 outputs: a few last-bit flips from delta's last bits


@pytest.mark.parametrize('hd,L,causal,order', [(64, 512, True, 'up'), (64, 512, False, 'up'), (96, 1024, True, 'up'),
                                                 (64, 520, False, 'perm'), (96, 300, True, 'perm')])
def test_attention_fwd_running_max_growth(hd, L, causal, order):
    """Scores that grow by far more than 2^16 (log2 units) from one key tile to the next: the forward's deferred running
    max must take its rescale path (recompute S, rescale O and the row sum) and still match fp32 softmax; 'perm' puts
    the large keys at random positions (growth at any tile, including inside the first). O and lse are checked (the
    backward recomputes P from lse)."""
    torch.manual_seed(hd + L)
    B, H = 2, 2
    d = H * hd
    q = (torch.rand(B, L, d, device=dev) * 0.5 + 0.75).bfloat16()           # positive: s grows with the key's norm
    mag = torch.linspace(0.0, 40.0, L, device=dev)
    if order == 'perm':
        mag = mag[torch.randperm(L, device=dev)]
    k = (torch.rand(B, L, d, device=dev) * 0.2 + mag[None, :, None]).bfloat16()
    v = torch.randn(B, L, d, device=dev).bfloat16()
    o = torch.empty(B, L, d, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    scale = hd ** -0.5
    K.attention(q, k, v, o, lse, B=B, H=H, Lq=L, Lk=L, hd=hd, sq=d, bq=L * d, sk=d, sv=d, bk=L * d, bv=L * d, so=d,
                bo=L * d, causal=causal)

    def heads(t):
        return t.float().view(B, L, H, hd).transpose(1, 2)

    s = heads(q) @ heads(k).transpose(-1, -2) * scale
    if causal:
        s = s.masked_fill(torch.ones(L, L, device=dev, dtype=torch.bool).triu(1), -float('inf'))
    ref = (s.softmax(-1) @ heads(v)).transpose(1, 2).reshape(B, L, d)
    assert _rel(o, ref) < 1e-2
    torch.testing.assert_close(lse, torch.logsumexp(s, -1), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize('B,H,L,hd,window,padded', [
    (2, 4, 512, 64, 4, True),       # the reference default (attn_window_size 4), C2 head dim
    (1, 2, 1024, 64, 4, False),     # band far from the [CLS] block
    (2, 2, 320, 96, 2, True),       # hd 96 (the 128-padded kernels)
    (1, 2, 640, 64, 1, False),      # window 1: diagonal block + [CLS] block only
    (2, 2, 256, 64, 8, False),      # window wider than the sequence: plain causal
    (1, 3, 1184, 32, 3, True),      # ragged tail (1184 = 37 blocks of 32), small head dim
    # the lengths the reference's sparse presets run (hparam_presets.py:122-171: 50 K / 100 K tokens per sample): past
    # 4096 padded keys the forward leaves the one-query-per-lane kernel for the 16x16 one (FWD32_MAXPAD), and the
    # backward's sliding-window key blocks sweep only their band (q_end) over 32 / 64 dQ planes
    (1, 2, 8192, 64, 4, True),
    (1, 2, 16384, 64, 4, True),
    (1, 2, 1024, 96, 4, True),      # hd 96 (two 256-key sub-blocks per plane): queries >= 640 through the [CLS] kernel
])
def test_attention_sliding_window_fwd_bwd(B, H, L, hd, window, padded):
    """window mode (SparseAttention's causal band + [CLS] block) vs a dense fp32 reference with the oracle's
    sparse mask; also the f32 kernel mode's forward. Past the band of dQ plane 0 (L >= 576 here) the [CLS] keys'
    share of the far queries runs in attn_bwd_cls_kernel (dK / dV through its f32 slabs)."""
    torch.manual_seed(L + window)
    d = H * hd
    q, k, v = (torch.randn(B, L, d, device=dev).bfloat16() for _ in range(3))
    pad = None
    if padded:
        pad = torch.zeros(B, L, device=dev, dtype=torch.uint8)
        for b in range(B):
            pad[b, L - 1 - 37 * b - 9:] = 1
    o = torch.empty(B, L, d, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    common = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=d, bq=L * d, sk=d, sv=d, bk=L * d, bv=L * d, so=d, bo=L * d,
                  key_pad=pad, causal=True, window=window)
    K.attention(q, k, v, o, lse, **common)

    def heads(t):
        return t.float().view(B, L, H, hd).transpose(1, 2)

    def unheads(t):
        return t.transpose(1, 2).reshape(B, L, d)

    qr, kr, vr = (heads(t).requires_grad_() for t in (q, k, v))
    s = qr @ kr.transpose(-1, -2) * hd ** -0.5
    mask = oracle.sparse_mask(L, window).to(dev)[None, None]
    if pad is not None:
        mask = mask | pad[:, None, None, :].bool()
    ref_o = unheads((s - mask * 1e7).softmax(-1) @ vr)
    assert _rel(o, ref_o) < 1e-2
    o32 = torch.empty(B, L, d, device=dev)
    K.attention_f32(q.float(), k.float(), v.float(), o32, **{kk: vv for kk, vv in common.items()})
    assert _rel(o32, ref_o) < 1e-5
    do = torch.randn(B, L, d, device=dev).bfloat16()
    ref_o.backward(do.float())
    dq = torch.full((B, L, d), 7.0, device=dev)    # every row written by the reduce
    dk = torch.empty(B, L, d, device=dev, dtype=torch.bfloat16)
    dv = torch.empty_like(dk)
    delta = torch.empty(B, H, L, device=dev)
    K.attention(q, k, v, o, lse, backward=True, dout=do, sdo=d, bdo=L * d, delta=delta, dq=dq, bdq=L * d,
                dk=dk, dv=dv, sdk=d, sdv=d, bdk=L * d, bdv=L * d, **common)
    assert _rel(dq, unheads(qr.grad)) < 2e-2
    assert _rel(dk, unheads(kr.grad)) < 2e-2
    assert _rel(dv, unheads(vr.grad)) < 2e-2


@pytest.mark.parametrize('B,H,L,hd', [
    (2, 4, 256, 64),     # every query < 256: dQ written final by key block 0 (no partial planes)
    (2, 2, 640, 96),     # hd 96: queries < 256 direct, the rest through the partial planes and the reduce
    (2, 2, 1100, 64),    # hd 64, two sub-blocks per plane: queries < 512 direct (with the first's partial added)
])
def test_attention_bwd_fused_dq_rotary(B, H, L, hd):
    """bf16 dQ with inverse rotary (from key block 0 directly, or from the partial-sum reduce) == f32 dQ followed by
    dq_finalize."""
    torch.manual_seed(9)
    d = H * hd
    qkv = torch.randn(B * L, 3 * d, device=dev).bfloat16()
    o = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    lse = torch.empty(B, H, L, device=dev)
    rot = rotary_table(L, d).to(dev)
    common = dict(B=B, H=H, Lq=L, Lk=L, hd=hd, sq=3 * d, bq=L * 3 * d, sk=3 * d, sv=3 * d, bk=L * 3 * d,
                  bv=L * 3 * d, so=d, bo=L * d, causal=True)
    K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, **common)
    do = torch.randn(B * L, d, device=dev).bfloat16()
    delta = torch.empty(B, H, L, device=dev)
    g32 = torch.empty(B * L, 3 * d, device=dev, dtype=torch.bfloat16)
    gbf = torch.empty_like(g32)
    dq = torch.empty(B * L, d, device=dev)
    bw = dict(backward=True, dout=do, sdo=d, bdo=L * d, delta=delta, sdk=3 * d, sdv=3 * d, bdk=L * 3 * d,
              bdv=L * 3 * d, rot=rot, rot_d=d)
    K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, dq=dq, bdq=L * d, dk=g32[:, d:], dv=g32[:, 2 * d:],
                **bw, **common)
    K.dq_finalize(dq, g32, 3 * d, B * L, d, rot, L)
    K.attention(qkv, qkv[:, d:], qkv[:, 2 * d:], o, lse, dq_bf=gbf, ldq_bf=3 * d, dk=gbf[:, d:], dv=gbf[:, 2 * d:],
                **bw, **common)
    torch.cuda.synchronize()
    assert _rel(gbf, g32.float()) < 1e-3


def test_attention_bwd_inverse_rotary_and_dq_finalize():
    torch.manual_seed(5)
    B, H, L, hd = 2, 2, 64, 64
    d = H * hd
    rot = rotary_table(L, d).to(dev)
    g = torch.randn(B * L, d, device=dev)
    out = torch.empty(B * L, d, device=dev, dtype=torch.bfloat16)
    K.dq_finalize(g, out, d, B * L, d, rot, L)
    # inverse rotary = gradient of the rotary map
    x = torch.randn(B, L, d).requires_grad_()
    oracle.rotary(x).backward(g.view(B, L, d).cpu())
    assert _rel(out.view(B, L, d).cpu(), x.grad) < 4e-3


def test_embedding_and_reparam():
    torch.manual_seed(6)
    V, D, T = 1000, 128, 300
    table = torch.randn(V, D, device=dev)
    ids = torch.randint(0, V, (T,), device=dev, dtype=torch.int32)
    out = torch.empty(T, D, device=dev)
    K.embedding_fwd(ids, table, out, T, D)
    assert torch.equal(out, table[ids.long()])
    dt = torch.zeros(V, D, device=dev)
    g = torch.randn(T, D, device=dev)
    K.embedding_bwd(ids, g, dt, T, D)
    ref = torch.zeros(V, D, device=dev).index_add_(0, ids.long(), g)
    assert _rel(dt, ref) < 1e-6
    B, Z = 5, 64
    stats = torch.randn(B, 2 * Z, device=dev) * 0.5
    eps = torch.randn(B, Z, device=dev)
    ntok = torch.tensor([100, 90, 80, 70, 60], device=dev)
    z, zb, eo, raw, kl = (torch.empty(B, Z, device=dev), torch.empty(B, Z, device=dev, dtype=torch.bfloat16),
                          torch.empty(B, Z, device=dev), torch.empty(B, device=dev), torch.empty(2, device=dev))
    K.reparam_fwd(stats, eps, 0, ntok, z, zb, eo, raw, kl, B, Z)
    s = stats.clone().requires_grad_()
    mu, lv = s[:, :Z], s[:, Z:]
    var = lv.exp()
    zr = mu + eps * var.sqrt()
    klr = 0.5 * (mu ** 2 + var - lv - 1.0)
    rawr = klr.sum(-1)
    assert _rel(z, zr) < 1e-6 and _rel(raw, rawr) < 1e-5
    assert abs(kl[0].item() - (rawr / ntok).mean().item()) < 1e-5 * abs(kl[0].item()) + 1e-7
    dz = torch.randn(B, Z, device=dev)
    (zr * dz).sum().add((rawr / ntok).mean() * 0.7).backward()
    gkl = torch.tensor([0.7], device=dev)
    ds = torch.empty(B, 2 * Z, device=dev)
    K.reparam_bwd(stats, eps, dz, ntok, gkl, ds, B, Z)
    assert _rel(ds, s.grad) < 1e-5
    # in-kernel noise: standard normal moments
    K.reparam_fwd(torch.zeros(64, 2 * Z, device=dev), None, 99, torch.ones(64, device=dev, dtype=torch.int64),
                  torch.empty(64, Z, device=dev), None, eo := torch.empty(64, Z, device=dev), torch.empty(64, device=dev),
                  torch.empty(2, device=dev), 64, Z)
    assert abs(eo.mean().item()) < 0.05 and abs(eo.std().item() - 1) < 0.05


def test_radam_kernel_matches_oracle():
    torch.manual_seed(7)
    n = 10000
    p = torch.randn(n, device=dev)
    m, v = torch.zeros(n, device=dev), torch.zeros(n, device=dev)
    pbf = torch.empty(n, device=dev, dtype=torch.bfloat16)
    st = oracle.RAdamState()
    ref = {'p': p.cpu().clone()}
    part = torch.empty(64, device=dev)
    norm = torch.empty(1, device=dev)
    for s in range(7):
        g = torch.randn(n, device=dev) * 3
        lr, b1, b2, eps, wd, max_norm = 1e-2, 0.9, 0.999, 1e-6, 0.01, 150.0
        step = st.step
        b2t = b2 ** step
        bcv = (1 - b2t) ** 0.5
        rho_inf = 2 / (1 - b2) - 1
        rho = rho_inf - 2 * step * b2t / (1 - b2t)
        lr_eff = lr
        if rho > 4:
            lr_eff = lr * (((rho - 4) * (rho - 2) * rho_inf) / ((rho_inf - 4) * (rho_inf - 2) * rho)) ** 0.5 * bcv
        scal = torch.tensor([lr_eff, 1 - b1 ** step, bcv, float(rho > 4), b1, b2, eps, wd, max_norm], device=dev)
        K.sumsq(g, n, part)
        K.radam(p, pbf, g, m, v, n, part, scal, norm)
        total, (gc,) = oracle.clip_grad_norm([g.cpu()], max_norm)
        ref = oracle.radam_step(ref, {'p': gc}, st, lr=lr, weight_decay=wd)
        assert abs(norm.item() - total.item()) / total.item() < 1e-5
        assert _rel(p, ref['p'].to(dev)) < 1e-6
    assert torch.equal(pbf, p.bfloat16())


def test_transpose_blocks_exact():
    g = torch.Generator(device=dev).manual_seed(3)
    src = torch.randn(200000, device=dev, generator=g).bfloat16()
    dst = torch.zeros_like(src)
    blocks = [(0, 192, 64), (20000, 1536, 72), (150000, 40, 1000)]   # (offset, rows, cols)
    tab, tiles = [], 0
    for o, r, c in blocks:
        tab.append([o, r, c, tiles])
        tiles += -(-r // 64) * -(-c // 64)
    K.transpose_blocks(src, dst, torch.tensor(tab, dtype=torch.int64, device=dev), len(blocks), tiles)
    torch.cuda.synchronize()
    for o, r, c in blocks:
        assert torch.equal(dst[o:o + r * c].view(c, r), src[o:o + r * c].view(r, c).t())


@pytest.mark.parametrize('D,p,with_x,with_z,with_ln,ydt', [(512, 0.1, True, True, True, 'f32'),
                                                           (768, 0.0, True, False, True, 'f32'),
                                                           (512, 0.3, True, False, False, 'bf16'),
                                                           (256, 0.0, False, False, True, 'bf16'),
                                                           (768, 0.25, True, True, True, 'bf16')])
def test_resid_ln_fwd(D, p, with_x, with_z, with_ln, ydt):
    """svae_resid_ln_fwd (the decoder's fused residual add + dropout + LayerNorm) against torch: v = x + dropout(y)
    with the mask of the counter RNG (recovered from dropout_bwd_cast of ones, the same index (r * D + c) / 4), the z
    rows on r % L == 0; xo bit-exact, LayerNorm 1e-2 rel in bf16, mean / rstd 1e-5."""
    torch.manual_seed(D + int(10 * p))
    L, B = 64, 6
    rows = B * L
    x = torch.randn(rows, D, device=dev) if with_x else None
    y = torch.randn(rows, D, device=dev)
    y = y.bfloat16() if ydt == 'bf16' else y
    zr = torch.randn(B, D, device=dev) if with_z else None
    w, b = 1 + 0.1 * torch.randn(D, device=dev), 0.1 * torch.randn(D, device=dev)
    seed = 12345 + D
    h = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    xo = torch.empty(rows, D, device=dev)
    mean, rstd = torch.empty(rows, device=dev), torch.empty(rows, device=dev)
    K.resid_ln_fwd(x, y, h, rows, D, w=w if with_ln else None, b=b if with_ln else None, mean=mean if with_ln else None,
                   rstd=rstd if with_ln else None, xo=xo, drop_p=p, seed=seed, zrows=zr, zmod=L if with_z else 0)
    keep = torch.empty(rows, D, device=dev, dtype=torch.bfloat16)
    K.dropout_bwd_cast(torch.ones(rows, D, device=dev), keep, p, seed, rows, D)
    yv = torch.where(keep.float() != 0, y.float() * (1.0 / (1.0 - p) if p > 0 else 1.0), torch.zeros_like(y.float()))
    v = (x if with_x else 0) + yv
    if with_z:
        v = v.view(B, L, D).clone()
        v[:, 0] = zr
        v = v.view(rows, D)
    assert torch.equal(xo, v)
    if with_ln:
        ref = torch.nn.functional.layer_norm(v, (D,), w, b, 1e-5)
        assert _rel(h, ref) < 1e-2
        torch.testing.assert_close(mean, v.mean(-1), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(rstd, (v.var(-1, unbiased=False) + 1e-5).rsqrt(), rtol=1e-4, atol=1e-5)
    else:
        assert torch.equal(h, v.bfloat16())


@pytest.mark.parametrize('M,Nn,Kk,hd,seq', [(24576, 512, 512, 64, 512),     # gemm256: the fused epilogue (hd 64)
                                            (16384, 768, 768, 96, 1024),    # gemm256, hd 96: heads across waves
                                            (4096, 512, 512, 64, 128),      # small grid: the separate delta kernel
                                            (64, 128, 128, 16, 1)])         # skinny GEMM, hd 16
def test_gemm_delta_epilogue(M, Nn, Kk, hd, seq):
    """svae_gemm's delta (the attention backward's rowsum(dO . O) per head, written by the dO GEMM): C identical to
    the plain BF16 GEMM, delta against torch on the bf16 C and the f32 O copy (summation order differs: 1e-5)."""
    torch.manual_seed(M + hd)
    A = torch.randn(M, Kk, device=dev).bfloat16()
    W = (torch.randn(Nn, Kk, device=dev) * 0.05).bfloat16()
    o32 = torch.randn(M, Nn, device=dev)
    C0 = torch.empty(M, Nn, device=dev, dtype=torch.bfloat16)
    K.gemm(A, W, C0, M, Nn, Kk, epi=N.EPI_BF16)
    C = torch.empty_like(C0)
    delta = torch.full((M * (Nn // hd),), 7.0, device=dev)
    K.gemm(A, W, C, M, Nn, Kk, epi=N.EPI_BF16, delta=delta, delta_o32=o32, ld_o32=Nn, delta_hd=hd, delta_seq=seq)
    torch.cuda.synchronize()
    assert torch.equal(C, C0)
    H = Nn // hd
    ref = (C.float() * o32).view(M // seq, seq, H, hd).sum(-1).permute(0, 2, 1).reshape(-1)
    torch.testing.assert_close(delta, ref, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize('nb', [5, 300])   # block table searched in LDS (<= 256 blocks) / in global memory
def test_transpose_blocks(nb):
    """svae_transpose_blocks (the transposed bf16 weight shadows): every block of the table transposed exactly, with
    ragged shapes (rows, cols multiples of 8, not of 64)."""
    g = torch.Generator().manual_seed(nb)
    shapes = [(8 * int(torch.randint(1, 40, (1,), generator=g)), 8 * int(torch.randint(1, 40, (1,), generator=g)))
              for _ in range(nb)]
    rows_tab, off, tiles = [], 0, 0
    for r, c in shapes:
        rows_tab.append((off, r, c, tiles))
        off += r * c
        tiles += -(-r // 64) * -(-c // 64)
    src = torch.randn(off, device=dev).bfloat16()
    dst = torch.zeros(off, device=dev, dtype=torch.bfloat16)
    table = torch.tensor(rows_tab, dtype=torch.int64, device=dev).flatten()
    K.transpose_blocks(src, dst, table, nb, tiles)
    torch.cuda.synchronize()
    for o, r, c, _ in rows_tab:
        assert torch.equal(dst[o:o + r * c].view(c, r), src[o:o + r * c].view(r, c).t())


def test_colsum_multi_exact():
    """svae_colsum_multi: up to 8 column sums in one launch, each added into its own output, exact on integer data
    (ragged row counts, the LayerNorm partial shape [nblk][2D] and narrower ones)."""
    g = torch.Generator(device=dev).manual_seed(7)
    segs, refs = [], []
    for rows, cols in ((1024, 1024), (1024, 1536), (37, 64), (513, 2048), (1, 4), (1024, 1024), (300, 128),
                       (1024, 1024)):
        inp = torch.randint(-3, 4, (rows, cols), device=dev, generator=g).float()
        out = torch.full((cols,), 0.5, device=dev)
        segs.append((inp, rows, cols, cols, out))
        refs.append(0.5 + inp.sum(0))
    K.colsum_multi(segs)
    torch.cuda.synchronize()
    for (_, _, _, _, out), ref in zip(segs, refs):
        assert torch.equal(out, ref)
