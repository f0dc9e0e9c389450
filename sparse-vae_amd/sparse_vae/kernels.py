"""Typed wrappers over libsvae.so (include/svae.h). Tensor in, pointer out; every wrapper checks the
arguments it relies on and raises on a non-zero status. All work is enqueued on torch's current HIP
stream; nothing here synchronises."""
import ctypes
import os

import torch

from . import _native as N
from ._native import lib, check, ptr, stream

bf16, f32 = torch.bfloat16, torch.float32

_gemm_desc = N.GemmDesc()


def _dev(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise RuntimeError('libsvae kernels need device tensors (no CPU fallback)')


def gemm(A, B, C, M, N_, K, *, a_t=False, b_t=False, lda=None, ldb=None, ldc=None, epi=N.EPI_BF16, bias=None,
         resid=None, ldr=0, aux=None, ldaux=0, alpha=1.0, splits=1, drop_p=0.0, seed=0, rot=None, rot_cols=0,
         rot_d=0, rot_seq=0, labels=None, label_logit=None, batch=1, sA=0, sB=0, sC=0, a_rowsum=None, k_weight=None,
         row_a=None, row_b=None, gather=None, ldg=0, delta=None, delta_o32=None, ld_o32=0, delta_hd=0, delta_seq=0):
    """C = epi(alpha * A . B) with A [M,K] (a_t: stored [K,M]) and B [K,N] (b_t: stored [K,N], else [N,K]).
    delta (BF16 epilogue): also the attention backward's delta = rowsum over each head of bf16(C) * delta_o32."""
    d = _fill_desc(_gemm_desc, A, B, C, M, N_, K, a_t=a_t, b_t=b_t, lda=lda, ldb=ldb, ldc=ldc, epi=epi, bias=bias,
                   resid=resid, ldr=ldr, aux=aux, ldaux=ldaux, alpha=alpha, splits=splits, drop_p=drop_p, seed=seed,
                   rot=rot, rot_cols=rot_cols, rot_d=rot_d, rot_seq=rot_seq, labels=labels, label_logit=label_logit,
                   batch=batch, sA=sA, sB=sB, sC=sC, a_rowsum=a_rowsum, k_weight=k_weight, row_a=row_a, row_b=row_b,
                   gather=gather, ldg=ldg)
    if delta is not None:
        _dev(delta, delta_o32)
        assert delta.dtype == f32 and delta_o32.dtype == f32 and delta.numel() >= M * (N_ // delta_hd)
    d.delta, d.delta_o32, d.ld_o32 = ptr(delta), ptr(delta_o32), ld_o32
    d.delta_hd, d.delta_seq = delta_hd, delta_seq
    check(lib.svae_gemm(ctypes.byref(d), stream()), 'svae_gemm')


def _fill_desc(d, A, B, C, M, N_, K, *, a_t=False, b_t=False, lda=None, ldb=None, ldc=None, epi=N.EPI_BF16,
               bias=None, resid=None, ldr=0, aux=None, ldaux=0, alpha=1.0, splits=1, drop_p=0.0, seed=0, rot=None,
               rot_cols=0, rot_d=0, rot_seq=0, labels=None, label_logit=None, batch=1, sA=0, sB=0, sC=0,
               a_rowsum=None, k_weight=None, row_a=None, row_b=None, gather=None, ldg=0):
    _dev(A, B, C)
    assert A.dtype == bf16 and B.dtype == bf16
    d.A, d.B = A.data_ptr(), B.data_ptr()
    d.lda = lda if lda is not None else (M if a_t else K)
    d.ldb = ldb if ldb is not None else (N_ if b_t else K)
    d.batch_stride_a, d.batch_stride_b = sA, sB
    d.M, d.N, d.K = M, N_, K
    d.batch, d.splits = batch, splits
    d.a_t, d.b_t = int(a_t), int(b_t)
    d.epi = epi
    d.C = ptr(C)          # None: CE statistics only (no logits stored)
    d.ldc = ldc if ldc is not None else N_
    d.batch_stride_c = sC
    d.bias = ptr(bias)
    d.resid = ptr(resid)
    d.ldr = ldr
    d.aux = ptr(aux)
    d.ldaux = ldaux
    d.alpha = alpha
    d.drop_p = drop_p
    d.seed = seed & 0xFFFFFFFFFFFFFFFF
    d.rot_tab = ptr(rot)
    d.rot_cols, d.rot_d, d.rot_seq = rot_cols, rot_d, rot_seq
    d.labels = ptr(labels)
    d.label_logit = ptr(label_logit)
    d.a_rowsum = ptr(a_rowsum)
    d.k_weight = ptr(k_weight)
    d.row_a, d.row_b = ptr(row_a), ptr(row_b)
    d.gather, d.ldg = ptr(gather), ldg
    d.delta, d.delta_o32, d.ld_o32, d.delta_hd, d.delta_seq = None, None, 0, 0, 0
    return d


_pair_desc = (N.GemmDesc(), N.GemmDesc())


def gemm_pair(g0, g1):
    """Two GEMMs in one launch (svae_gemm_pair): g0, g1 are (args, kwargs) of gemm() for two split-K slab weight
    gradients (a_t, b_t, epi F32_ATOMIC, splits >= 2, aux = slab workspace)."""
    d0 = _fill_desc(_pair_desc[0], *g0[0], **g0[1])
    d1 = _fill_desc(_pair_desc[1], *g1[0], **g1[1])
    check(lib.svae_gemm_pair(ctypes.byref(d0), ctypes.byref(d1), stream()), 'svae_gemm_pair')


def auto_splits(M, N_, K, target=512):
    """Split-K count for a dW GEMM. First choice: one round of 192..256 blocks of the 256x256 kernel (the
    library picks it at >= 192 blocks); otherwise ~`target` blocks of the 128x128 kernels."""
    t256 = -(-M // 256) * -(-N_ // 256)
    if t256 >= 192:
        return 1
    if t256 >= 4:   # fill the 256 CUs with one round of 256x256 blocks (1 per CU), K-slices >= 512
        # (the 512 x 512 dW over 32768 rows with bias row sums: 64 x 256^2 slices 50.7 us against 62.3 us for
        # 32 x 128^2 -- scripts/dw_split_probe.py with DW_RS=1, profiles/r02_dw_split_impl.log)
        s3 = min(256 // t256, max(1, K // 512))
        if t256 * s3 >= 192:
            return s3
    tiles = -(-M // 128) * -(-N_ // 128)
    if tiles >= 256 or K < 1024:
        return 1
    s = min(-(-target // tiles), K // 512)
    return max(1, s)


def linear_dw(dY, X, Wgrad, rows, n_out, n_in, ldy=None, ldx=None, bgrad=None):
    """Wgrad[n_out, n_in] += dY^T . X over `rows` rows (dY [rows, n_out] bf16, X [rows, n_in] bf16); with
    bgrad, also bgrad[n_out] += column sums of dY (the bias gradient, fused into the same pass over dY)."""
    s = auto_splits(n_out, n_in, rows)
    slab = _slab_workspace(s * n_out * n_in, dY.device) if s > 1 else None
    gemm(dY, X, Wgrad, n_out, n_in, rows, a_t=True, b_t=True, lda=ldy or n_out, ldb=ldx or n_in, ldc=n_in,
         epi=N.EPI_F32_ATOMIC if s > 1 else N.EPI_F32_ACC, splits=s, a_rowsum=bgrad, aux=slab)


def pair_splits(shapes):
    """Split-K counts (s0, s1) for two weight gradients launched together ((n_out, n_in, rows) each): one round of
    <= 256 256x256 blocks over both, every block's K-slice about the same length (rows / s, >= 512 rows), so a GEMM
    over many more rows than its partner is split further (C2's encoder pair of a 4096-row and a 32768-row dW: 4 and
    30 splits, 256 blocks, instead of 8 and 8, 96 blocks of which 64 ran 64 K-tiles). None when either would not
    split (then run them apart). SVAE_DW_PAIR_EQUAL=1: one common count (the round-3 rule), for A/B."""
    tiles = [-(-m // 256) * -(-n // 256) for m, n, _ in shapes]
    rows = [r for _, _, r in shapes]
    if not all(tiles):
        return None
    if os.environ.get('SVAE_DW_PAIR_EQUAL', '0') != '0':
        c = min([256 // sum(tiles)] + [r // 512 for r in rows])
        return (c, c) if c >= 2 else None
    cap = [r // 512 for r in rows]
    if min(cap) < 2:
        return None
    work = sum(t * r for t, r in zip(tiles, rows))
    slice_rows = max(512.0, work / 256.0)
    sp = [min(c, max(2, round(r / slice_rows))) for r, c in zip(rows, cap)]
    while sum(t * x for t, x in zip(tiles, sp)) > 256:
        # shorten the longest per-block slice's partner: drop a split where the slice is shortest
        i = min((k for k in range(2) if sp[k] > 2), key=lambda k: rows[k] / sp[k], default=None)
        if i is None:
            return None
        sp[i] -= 1
    # the kernel's K-slice is a multiple of 64 rows: count only the non-empty slices
    sp = [-(-r // (-(-(-(-r // x)) // 64) * 64)) for r, x in zip(rows, sp)]
    longest = max(r / x for r, x in zip(rows, sp))
    for k in range(2):   # no more slabs than the longest slice needs
        while sp[k] > 2 and rows[k] / (sp[k] - 1) <= longest:
            sp[k] -= 1
    return tuple(sp)


def linear_dw_pair(j0, j1):
    """Two linear_dw's (each (dY, X, Wgrad, rows, n_out, n_in, ldy, ldx, bgrad)) as one paired launch: each needs
    only ~half the split-K slices it would take alone to fill the chip (half the slab bytes written and reduced).
    Falls back to two linear_dw calls for shapes that would not split."""
    sp = pair_splits([(j[4], j[5], j[3]) for j in (j0, j1)])
    if sp is None:
        linear_dw(*j0[:8], bgrad=j0[8])
        linear_dw(*j1[:8], bgrad=j1[8])
        return
    n0, n1 = sp[0] * j0[4] * j0[5], sp[1] * j1[4] * j1[5]
    slab = _slab_workspace(n0 + n1, j0[0].device)
    gs = []
    for j, aux, s in ((j0, slab[:n0], sp[0]), (j1, slab[n0:n0 + n1], sp[1])):
        dY, X, Wg, rows, n_out, n_in, ldy, ldx, bg = j
        gs.append(((dY, X, Wg, n_out, n_in, rows),
                   dict(a_t=True, b_t=True, lda=ldy or n_out, ldb=ldx or n_in, ldc=n_in, epi=N.EPI_F32_ATOMIC,
                        splits=s, a_rowsum=bg, aux=aux)))
    gemm_pair(*gs)


_slabs = {}


def _slab_workspace(n, device):
    """f32 split-K slab workspace (grown on demand, reused stream-ordered by every dW GEMM)."""
    t = _slabs.get(device)
    if t is None or t.numel() < n:
        t = torch.empty(n, dtype=torch.float32, device=device)
        _slabs[device] = t
    return t


def resid_ln_fwd(x, y, h, rows, D, *, w=None, b=None, mean=None, rstd=None, xo=None, drop_p=0.0, seed=0, zrows=None,
                 zmod=0):
    """svae_resid_ln_fwd: v = x + dropout(y) (or zrows[r // zmod] on rows r % zmod == 0); xo = v; h = LN(v) (or bf16(v)
    without w / b)."""
    _dev(h, *(t for t in (x, y, xo, zrows, w, b, mean, rstd) if t is not None))
    assert h.dtype == bf16 and (y is None or y.dtype in (bf16, f32)) and (x is None or x.dtype == f32)
    # the kernel walks x / xo / zrows / h as dense rows of D elements (y has its own leading dimension)
    for t in (x, xo, zrows, h, w, b):
        assert t is None or t.is_contiguous(), 'resid_ln_fwd: x, xo, zrows, h, w, b must be contiguous'
    check(lib.svae_resid_ln_fwd(ptr(x), ptr(y), 1 if y is not None and y.dtype == bf16 else 0,
                                y.stride(0) if y is not None else 0, float(drop_p), int(seed) & (2 ** 64 - 1),
                                ptr(zrows), int(zmod), ptr(w), ptr(b), ptr(xo), h.data_ptr(), ptr(mean), ptr(rstd), rows,
                                D, stream()), 'svae_resid_ln_fwd')


def layernorm_fwd(x, w, b, y, mean, rstd, rows, D):
    _dev(x, w, b, y, mean, rstd)
    check(lib.svae_layernorm_fwd(x.data_ptr(), 0 if x.dtype == f32 else 1, w.data_ptr(), b.data_ptr(), y.data_ptr(),
                                 mean.data_ptr(), rstd.data_ptr(), rows, D, stream()), 'svae_layernorm_fwd')


def layernorm_bwd(dy, x, w, mean, rstd, dres, dx, dx_bf, wgrad2, rows, D, part_ws, bf_drop=None, zsplice=None,
                  defer=None):
    """dx = dres + LN'(dy); wgrad2 (the adjacent [weight | bias] grads, 2D floats) += sum of affine grads.
    bf_drop = (p, seed, zero_mod): the bf16 copy dx_bf carries the next consumer's dropout backward and position-0
    zeroing (svae_layernorm_bwd_drop), replacing a dropout_bwd_cast pass over dx. zsplice = (L, zrow f32 | None,
    zrow_bf bf16 | None): rows r % L == 0 of dx go to zrow[r / L] / zrow_bf and are zeroed in dx (extract_rows)."""
    nblk = lib.svae_layernorm_nblk(rows)
    part = part_ws[: nblk * 2 * D]
    if bf_drop is None and zsplice is None:
        check(lib.svae_layernorm_bwd(dy.data_ptr(), x.data_ptr(), 0 if x.dtype == f32 else 1, w.data_ptr(),
                                     mean.data_ptr(), rstd.data_ptr(), ptr(dres), dx.data_ptr(), ptr(dx_bf),
                                     part.data_ptr(), nblk, rows, D, 0, stream()), 'svae_layernorm_bwd')
    else:
        p, seed, zmod = bf_drop if bf_drop is not None else (0.0, 0, 0)
        zm, zrow, zrow_bf = zsplice if zsplice is not None else (0, None, None)
        check(lib.svae_layernorm_bwd_drop(dy.data_ptr(), x.data_ptr(), 0 if x.dtype == f32 else 1, w.data_ptr(),
                                          mean.data_ptr(), rstd.data_ptr(), ptr(dres), dx.data_ptr(), ptr(dx_bf),
                                          part.data_ptr(), nblk, rows, D, int(zm), float(p),
                                          int(seed) & 0xFFFFFFFFFFFFFFFF, int(zmod), ptr(zrow), ptr(zrow_bf),
                                          stream()), 'svae_layernorm_bwd_drop')
    if defer is not None:   # the caller sums the partials later, batched with other LayerNorms (colsum_multi)
        defer.append((part, nblk, 2 * D, 2 * D, wgrad2))
    else:
        colsum(part, nblk, 2 * D, 2 * D, wgrad2, accumulate=True)


def layernorm_bwd_gelu(dy, x, w, mean, rstd, gp, out_bf, wgrad2, rows, D, part_ws, defer=None):
    """out_bf = bf16(LN'(dy) * gp) (svae_layernorm_bwd_gelu: the head's LayerNorm backward with the GELU backward
    of the linear before it); wgrad2 += the affine grads (or deferred, as layernorm_bwd)."""
    nblk = lib.svae_layernorm_nblk(rows)
    part = part_ws[: nblk * 2 * D]
    check(lib.svae_layernorm_bwd_gelu(dy.data_ptr(), x.data_ptr(), 0 if x.dtype == f32 else 1, w.data_ptr(),
                                      mean.data_ptr(), rstd.data_ptr(), gp.data_ptr(), out_bf.data_ptr(),
                                      part.data_ptr(), nblk, rows, D, stream()), 'svae_layernorm_bwd_gelu')
    if defer is not None:
        defer.append((part, nblk, 2 * D, 2 * D, wgrad2))
    else:
        colsum(part, nblk, 2 * D, 2 * D, wgrad2, accumulate=True)


def _ptrs(ts):
    return (ctypes.c_void_p * N.LN_MULTI_MAX)(*[t.data_ptr() for t in ts])


def layernorm_fwd_multi(x, ws, bs, ys, mean, rstd, rows, D):
    """svae_layernorm_fwd_multi: ys[j] = bf16(LN(x) * ws[j] + bs[j]) for n <= LN_MULTI_MAX affines of one f32 x
    (the encoder middle layers' context LayerNorms), one pass; the shared mean / rstd."""
    n = len(ys)
    assert 0 < n <= N.LN_MULTI_MAX and len(ws) == n and len(bs) == n and x.dtype == f32
    _dev(x, mean, rstd, *ws, *bs, *ys)
    check(lib.svae_layernorm_fwd_multi(x.data_ptr(), _ptrs(ws), _ptrs(bs), _ptrs(ys), n, mean.data_ptr(),
                                       rstd.data_ptr(), rows, D, stream()), 'svae_layernorm_fwd_multi')


def layernorm_bwd_multi(dys, x, ws, mean, rstd, dres, dx, wgrads, rows, D, part_ws, defer=None):
    """svae_layernorm_bwd_multi: dx = dres + sum_j LN'_j(dys[j]) (dres may be dx); wgrads[j] (the adjacent
    [weight | bias] grads of LayerNorm j) += its affine grads, summed from part_ws (n slabs) now or by the caller's
    deferred colsum_multi (defer, as layernorm_bwd)."""
    n = len(dys)
    assert 0 < n <= N.LN_MULTI_MAX and len(ws) == n and len(wgrads) == n and x.dtype == f32
    _dev(x, mean, rstd, dx, *dys, *ws)
    nblk = lib.svae_layernorm_nblk(rows)
    parts = [part_ws[j * nblk * 2 * D:(j + 1) * nblk * 2 * D] for j in range(n)]
    assert parts[-1].numel() == nblk * 2 * D
    check(lib.svae_layernorm_bwd_multi(_ptrs(dys), x.data_ptr(), _ptrs(ws), mean.data_ptr(), rstd.data_ptr(),
                                       ptr(dres), dx.data_ptr(), _ptrs(parts), nblk, n, rows, D, stream()),
          'svae_layernorm_bwd_multi')
    for part, wg in zip(parts, wgrads):
        if defer is not None:
            defer.append((part, nblk, 2 * D, 2 * D, wg))
        else:
            colsum(part, nblk, 2 * D, 2 * D, wg, accumulate=True)


_colsum_segs = (N.ColsumSeg * N.COLSUM_MAX)()


def colsum_multi(segs):
    """svae_colsum_multi: [(inp f32, rows, cols, ld, out f32)] (<= 8), each out += column sums of its inp."""
    assert 0 < len(segs) <= N.COLSUM_MAX
    for i, (inp, rows, cols, ld, out) in enumerate(segs):
        _dev(inp, out)
        assert inp.dtype == f32 and out.dtype == f32
        _colsum_segs[i].inp, _colsum_segs[i].out = inp.data_ptr(), out.data_ptr()
        _colsum_segs[i].ld, _colsum_segs[i].rows, _colsum_segs[i].cols = ld, rows, cols
    check(lib.svae_colsum_multi(ctypes.addressof(_colsum_segs), len(segs), stream()), 'svae_colsum_multi')


def colsum(inp, rows, cols, ld, out, accumulate=True):
    check(lib.svae_colsum(inp.data_ptr(), 0 if inp.dtype == f32 else 1, rows, cols, ld, out.data_ptr(),
                          int(accumulate), stream()), 'svae_colsum')


_attn_desc = N.AttnDesc()


def attention(q, k, v, o, lse, *, B, H, Lq, Lk, hd, sq, sk, sv, so, bq, bk, bv, bo, key_pad=None, causal=False,
              window=0, scale=None, backward=False, dout=None, sdo=0, bdo=0, delta=None, dq=None, bdq=0, dk=None, dv=None,
              sdk=0, sdv=0, bdk=0, bdv=0, rot=None, rot_d=0, o32=None, so32=0, bo32=0, dq_part=None, dq_bf=None,
              ldq_bf=0, delta_ready=False, o_lo=None, so_lo=0, bo_lo=0):
    """Forward (o, lse[, o32 | o_lo]) or backward (dk, dv and dq: f32 `dq` or bf16 `dq_bf` with inverse rotary).
    o_lo: bf16 residual O - bf16(O) (written by the forward, read by the backward's delta pass; the 2-byte alternative
    to the f32 copy o32).
    dq_part: f32 workspace of attn_dq_part_elems(...) floats (allocated here when not given).
    window > 0 (causal): SparseAttention's sliding window of `window` 32-key blocks + the [CLS] block."""
    d = _attn_desc
    d.q, d.k, d.v, d.o = q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr()
    d.sq, d.sk, d.sv, d.so, d.bq, d.bk, d.bv, d.bo = sq, sk, sv, so, bq, bk, bv, bo
    d.key_pad = ptr(key_pad)
    d.lse = lse.data_ptr()
    d.B, d.H, d.Lq, d.Lk, d.hd, d.causal = B, H, Lq, Lk, hd, int(causal)
    d.window = int(window)
    d.delta_ready = int(bool(delta_ready))
    d.scale = hd ** -0.5 if scale is None else scale
    d.o32, d.so32, d.bo32 = ptr(o32), so32, bo32
    d.o_lo, d.so_lo, d.bo_lo = ptr(o_lo), so_lo, bo_lo
    if backward:
        d.fwd_ws, d.fwd_ws_elems = None, 0
        d.dout, d.sdo, d.bdo = dout.data_ptr(), sdo, bdo
        d.delta, d.bdq = delta.data_ptr(), bdq
        d.dk, d.dv, d.sdk, d.sdv, d.bdk, d.bdv = dk.data_ptr(), dv.data_ptr(), sdk, sdv, bdk, bdv
        d.rot_tab, d.rot_d = ptr(rot), rot_d
        if dq_part is None:
            dq_part = torch.empty(attn_dq_part_elems(B, H, Lq, Lk, hd, window), device=q.device, dtype=torch.float32)
        assert dq_part.numel() >= attn_dq_part_elems(B, H, Lq, Lk, hd, window) and dq_part.dtype == torch.float32
        d.dq_part, d.dq_bf, d.ldq_bf = dq_part.data_ptr(), ptr(dq_bf), ldq_bf
        d.dq = ptr(dq)
        check(lib.svae_attn_bwd(ctypes.byref(d), stream()), 'svae_attn_bwd')
    else:
        d.dout = None
        # few queries over a long key sequence: the split-KV workspace (the library decides; 0 floats = one pass)
        n = lib.svae_attn_fwd_ws_elems(B, H, Lq, Lk, hd, int(causal), int(window))
        if n > 0:
            ws = _fwd_workspace(n, q.device)
            d.fwd_ws, d.fwd_ws_elems = ws.data_ptr(), ws.numel()
        else:
            d.fwd_ws, d.fwd_ws_elems = None, 0
        check(lib.svae_attn_fwd(ctypes.byref(d), stream()), 'svae_attn_fwd')


_fwd_ws = {}


def _fwd_workspace(n, device):
    """f32 workspace of the split-KV attention forward (grown on demand, reused stream-ordered)."""
    t = _fwd_ws.get(device)
    if t is None or t.numel() < n:
        t = torch.empty(n, dtype=torch.float32, device=device)
        _fwd_ws[device] = t
    return t


def attn_dq_part_elems(B, H, Lq, Lk, hd, window=0):
    """Floats of the backward's dQ-partial workspace for this shape (window > 0: the sliding window's compact band
    planes)."""
    return lib.svae_attn_dq_part_elems_w(B, H, Lq, Lk, hd, int(window))


def dq_finalize(dq, out, ldo, rows, D, rot=None, seq=0):
    check(lib.svae_dq_finalize(dq.data_ptr(), out.data_ptr(), ldo, rows, D, ptr(rot), seq, stream()),
          'svae_dq_finalize')


def embedding_fwd(ids, table, out, rows, D, out2=None):
    if out2 is not None:
        _dev(ids, table, out, out2)
        check(lib.svae_embedding_fwd_dual(ids.data_ptr(), table.data_ptr(), out.data_ptr(), out2.data_ptr(), rows, D,
                                          stream()), 'svae_embedding_fwd_dual')
        return
    check(lib.svae_embedding_fwd(ids.data_ptr(), table.data_ptr(), out.data_ptr(), None, rows, D, stream()),
          'svae_embedding_fwd')


def embedding_bwd(ids, dout, dtable, rows, D):
    check(lib.svae_embedding_bwd(ids.data_ptr(), dout.data_ptr(), dtable.data_ptr(), rows, D, stream()),
          'svae_embedding_bwd')


def reparam_fwd(stats, eps, seed, ntok, z, z_bf, eps_out, raw_kl, kl_out, B, Z):
    check(lib.svae_reparam_kl_fwd(stats.data_ptr(), ptr(eps), seed & 0xFFFFFFFFFFFFFFFF, ntok.data_ptr(),
                                  z.data_ptr(), ptr(z_bf), ptr(eps_out), raw_kl.data_ptr(), kl_out.data_ptr(), B, Z,
                                  stream()), 'svae_reparam_kl_fwd')


def reparam_bwd(stats, eps, dz, ntok, gkl, dstats, B, Z):
    check(lib.svae_reparam_kl_bwd(stats.data_ptr(), eps.data_ptr(), ptr(dz), ntok.data_ptr(), gkl.data_ptr(),
                                  dstats.data_ptr(), B, Z, stream()), 'svae_reparam_kl_bwd')


def ce_red_ws(device, nchunks):
    """f32 workspace of the chunked-CE reductions (grown on demand)."""
    n = max(1024, lib.svae_ce_red_ws_elems(nchunks))
    t = _ce_red.get(device)
    if t is None or t.numel() < n:
        t = _ce_red[device] = torch.empty(n, dtype=f32, device=device)
    return t


_ce_red = {}


def ce_finalize(part, ntile, label_logit, labels, rows, seq, nchunks, chunk_len, lse, row_loss, chunk_w, nll):
    assert chunk_w.numel() >= nchunks and chunk_w.dtype == f32
    red = ce_red_ws(part.device, nchunks)
    check(lib.svae_ce_finalize(part.data_ptr(), ntile, label_logit.data_ptr(), labels.data_ptr(), rows, seq,
                               nchunks, chunk_len, lse.data_ptr(), row_loss.data_ptr(), chunk_w.data_ptr(),
                               nll.data_ptr(), red.data_ptr(), stream()), 'svae_ce_finalize')


def ce_weighted_nll(row_loss, labels, tok_w, rows, seq, nchunks, chunk_len, out):
    """Chunked mean of row_loss with per-target weights tok_w [V] (F.cross_entropy(weight=...)), into out[0]."""
    _dev(row_loss, labels, tok_w, out)
    assert tok_w.dtype == f32 and tok_w.is_contiguous()
    red = ce_red_ws(row_loss.device, nchunks)
    check(lib.svae_ce_weighted_nll(row_loss.data_ptr(), labels.data_ptr(), tok_w.data_ptr(), rows, seq, nchunks,
                                   chunk_len, out.data_ptr(), red.data_ptr(), stream()), 'svae_ce_weighted_nll')


def ce_chunking(B, L, V, chunk_numel=2 ** 30):
    """robust_cross_entropy's split (language_model.py:163-170) of logits [B, L-1, V]: cdiv(numel, 2^30) chunks
    requested along the sequence; torch.chunk makes ceil((L-1)/chunks)-long pieces, so fewer may result.
    Returns (nchunks, chunk_len)."""
    chunks = -(-(B * (L - 1) * V) // chunk_numel)
    chunk_len = -(-(L - 1) // chunks)
    return -(-(L - 1) // chunk_len), chunk_len


def ce_label_logit(hh, W, bias, labels, rows, D, out):
    _dev(hh, W, labels, out)
    check(lib.svae_ce_label_logit(hh.data_ptr(), hh.stride(0), W.data_ptr(), W.stride(0), ptr(bias), labels.data_ptr(),
                                  rows, D, out.data_ptr(), stream()), 'svae_ce_label_logit')


def ce_prob_finalize(part, ntile, row_off, labels, rows, seq, nchunks, chunk_len, lse, row_loss, chunk_w, nll,
                     fix=None):
    """fix = (hh, W, bias, P, sat_ws): recompute the rows whose P saturated (svae_ce_prob_finalize_fix); sat_ws
    int32 [1 + rows] holds their count (and rows) afterwards."""
    assert chunk_w.numel() >= nchunks and chunk_w.dtype == f32
    red = ce_red_ws(part.device, nchunks)
    if fix is None:
        check(lib.svae_ce_prob_finalize(part.data_ptr(), ntile, row_off.data_ptr(), labels.data_ptr(), rows, seq,
                                        nchunks, chunk_len, lse.data_ptr(), row_loss.data_ptr(), chunk_w.data_ptr(),
                                        nll.data_ptr(), red.data_ptr(), stream()), 'svae_ce_prob_finalize')
        return
    hh, W, bias, P, sat = fix
    _dev(hh, W, P, sat)
    assert sat.dtype == torch.int32 and sat.numel() >= rows + 1 and P.shape[0] >= rows
    check(lib.svae_ce_prob_finalize_fix(part.data_ptr(), ntile, row_off.data_ptr(), labels.data_ptr(), rows, seq,
                                        nchunks, chunk_len, lse.data_ptr(), row_loss.data_ptr(), chunk_w.data_ptr(),
                                        nll.data_ptr(), red.data_ptr(), hh.data_ptr(), hh.stride(0), W.data_ptr(),
                                        W.stride(0), ptr(bias), P.data_ptr(), P.stride(0), W.shape[0], hh.shape[1],
                                        sat.data_ptr(), stream()), 'svae_ce_prob_finalize_fix')


def ce_prob_bwd_prep(hh, lse, row_off, chunk_w, labels, gscale, rows, seq, nchunks, chunk_len, D, hh_out, r_out,
                     q_out, dbias=None):
    _dev(hh, lse, row_off, chunk_w, labels, gscale, hh_out, r_out, q_out)
    check(lib.svae_ce_prob_bwd_prep(hh.data_ptr(), hh.stride(0), lse.data_ptr(), row_off.data_ptr(),
                                    chunk_w.data_ptr(), labels.data_ptr(), gscale.data_ptr(), rows, seq, nchunks,
                                    chunk_len, D, hh_out.data_ptr(), r_out.data_ptr(), q_out.data_ptr(), ptr(dbias),
                                    stream()), 'svae_ce_prob_bwd_prep')


def embedding_bwd_ce(ids, dout, dtable, rows, D, seq, hh, q):
    check(lib.svae_embedding_bwd_ce(ids.data_ptr(), dout.data_ptr(), dtable.data_ptr(), rows, D, seq, hh.data_ptr(),
                                    q.data_ptr(), stream()), 'svae_embedding_bwd_ce')


def mutual_info(stats, kl, B, Z, seed, out, ws, eps=None, S=10):
    """out[0] = kl[0] - marginal_kl (math_utils.py:51-58) over S posterior samples; eps [S, B, Z] or in-kernel."""
    _dev(stats, kl, out, ws)
    assert ws.numel() >= 2 * S * B
    check(lib.svae_mutual_info(stats.data_ptr(), ptr(eps), seed & 0xFFFFFFFFFFFFFFFF, kl.data_ptr(), B, Z, S,
                               ws.data_ptr(), out.data_ptr(), stream()), 'svae_mutual_info')


def ce_seq_logprob(part, ntile, label_logit, labels, rows, seq, out):
    _dev(part, label_logit, labels, out)
    assert out.dtype == f32 and out.numel() == rows // seq and out.is_contiguous()
    check(lib.svae_ce_seq_logprob(part.data_ptr(), ntile, label_logit.data_ptr(), labels.data_ptr(), rows, seq,
                                  out.data_ptr(), stream()), 'svae_ce_seq_logprob')


def ce_grad(logits, ld, lse, chunk_w, labels, gscale, rows, V, seq, nchunks, chunk_len, dbias=None):
    check(lib.svae_ce_grad(logits.data_ptr(), ld, lse.data_ptr(), chunk_w.data_ptr(), labels.data_ptr(),
                           gscale.data_ptr(), ptr(dbias), rows, V, seq, nchunks, chunk_len, stream()), 'svae_ce_grad')


def prep_tokens(ids, pad, B, L, ids32, labels, padm=None, ntok=None, ntok_out=None):
    """svae_prep_tokens: ids int64 [B, L] -> ids32, next-token labels (0 at each sequence's end), the uint8
    padding mask (pad True: ids == 0; a bool tensor: copied; None / False: none) and the ntok copy."""
    assert ids.dtype == torch.int64 and ids.is_contiguous() and ids.numel() == B * L
    mode = 0 if pad is None or pad is False else (1 if pad is True else 2)
    if mode == 2:
        assert pad.dtype == torch.bool and pad.is_contiguous() and pad.numel() == B * L
    if ntok is not None:
        assert ntok.dtype == torch.int64 and ntok.is_contiguous() and ntok.numel() == B
    _dev(ids, ids32, labels)
    check(lib.svae_prep_tokens(ids.data_ptr(), pad.data_ptr() if mode == 2 else None, mode, B, L, ids32.data_ptr(),
                               labels.data_ptr(), ptr(padm), ptr(ntok), ptr(ntok_out), stream()), 'svae_prep_tokens')


def step_scalars(kl_weight, nll=None, kl=None, loss=None, gloss=None, gs=None):
    """svae_step_scalars: loss = nll + kl_weight * kl and / or gs = (gloss, gloss * kl_weight), f32 on the device."""
    for t in (nll, kl, loss, gloss, gs):
        assert t is None or (t.is_cuda and t.dtype == f32)
    check(lib.svae_step_scalars(ptr(nll), ptr(kl), ptr(gloss), float(kl_weight), ptr(loss), ptr(gs), stream()),
          'svae_step_scalars')


def dropout_bwd_cast(g, out, p, seed, rows, cols, ld_in=None):
    check(lib.svae_dropout_bwd_cast(g.data_ptr(), out.data_ptr(), p, seed & 0xFFFFFFFFFFFFFFFF, rows * cols, cols,
                                    ld_in or cols, stream()), 'svae_dropout_bwd_cast')


def cast_bf16(x, out, n=None):
    check(lib.svae_cast_bf16(x.data_ptr(), out.data_ptr(), n if n is not None else x.numel(), stream()),
          'svae_cast_bf16')


def transpose_blocks(src, dst, table, nblocks, total_tiles):
    check(lib.svae_transpose_blocks(src.data_ptr(), dst.data_ptr(), table.data_ptr(), nblocks, total_tiles, stream()),
          'svae_transpose_blocks')


def gelu_bwd(dx, gp, out, n):
    check(lib.svae_gelu_bwd(dx.data_ptr(), gp.data_ptr(), out.data_ptr(), n, stream()), 'svae_gelu_bwd')


def extract_rows(x, ld, rows, mod, D, out):
    check(lib.svae_extract_rows(x.data_ptr(), ld, rows, mod, D, out.data_ptr(), stream()), 'svae_extract_rows')


def zproj_bwd(g, z, W, dW, db, dz, B, d, Z):
    """z_projections backward (svae_zproj_bwd): dW += g^T z, db += sum_b g, dz += g W (g f32 [B, d]; z, W bf16)."""
    _dev(g, z, W, dW, db, dz)
    assert g.dtype == f32 and z.dtype == bf16 and W.dtype == bf16 and dW.dtype == f32 and dz.dtype == f32
    check(lib.svae_zproj_bwd(g.data_ptr(), z.data_ptr(), W.data_ptr(), dW.data_ptr(), db.data_ptr(), dz.data_ptr(),
                             B, d, Z, stream()), 'svae_zproj_bwd')


_zfwd_segs = (N.ZprojFwdSeg * N.ZPROJ_MAX)()


def zproj_fwd_multi(segs, z, B, d, Z):
    """svae_zproj_fwd_multi: segs = [(W bf16 [d, Z], bias f32 [d], out f32 [B, d])] (<= 32): out = z W^T + bias."""
    assert 0 < len(segs) <= N.ZPROJ_MAX
    _dev(z)
    assert z.dtype == bf16 and z.is_contiguous()
    for i, (W, bias, out) in enumerate(segs):
        _dev(W, bias, out)
        assert W.dtype == bf16 and bias.dtype == f32 and out.dtype == f32 and out.is_contiguous()
        _zfwd_segs[i].W, _zfwd_segs[i].bias, _zfwd_segs[i].out = W.data_ptr(), bias.data_ptr(), out.data_ptr()
    check(lib.svae_zproj_fwd_multi(ctypes.addressof(_zfwd_segs), len(segs), z.data_ptr(), B, d, Z, stream()),
          'svae_zproj_fwd_multi')


def layernorm_fwd_z(x, zrows, zmod, w, b, y, mean, rstd, rows, D):
    """svae_layernorm_fwd_z: LayerNorm forward of f32 x whose rows r % zmod == 0 come from zrows (and are written into x)."""
    _dev(x, zrows, w, b, y, mean, rstd)
    assert x.dtype == f32 and zrows.dtype == f32 and x.is_contiguous() and zrows.is_contiguous()
    check(lib.svae_layernorm_fwd_z(x.data_ptr(), zrows.data_ptr(), zmod, w.data_ptr(), b.data_ptr(), y.data_ptr(),
                                   mean.data_ptr(), rstd.data_ptr(), rows, D, stream()), 'svae_layernorm_fwd_z')


_zproj_segs = (N.ZprojSeg * N.ZPROJ_MAX)()


def zproj_bwd_multi(segs, z, dz, B, d, Z):
    """svae_zproj_bwd_multi: segs = [(g f32 [B, d], W bf16 [d, Z], dW f32, db f32)] (<= 32) sharing z and dz; the
    same results as zproj_bwd per segment in list order."""
    assert 0 < len(segs) <= N.ZPROJ_MAX
    _dev(z, dz)
    assert z.dtype == bf16 and dz.dtype == f32
    for i, (g, W, dW, db) in enumerate(segs):
        _dev(g, W, dW, db)
        assert g.dtype == f32 and W.dtype == bf16 and dW.dtype == f32 and db.dtype == f32
        _zproj_segs[i].g, _zproj_segs[i].W = g.data_ptr(), W.data_ptr()
        _zproj_segs[i].dW, _zproj_segs[i].db = dW.data_ptr(), db.data_ptr()
    check(lib.svae_zproj_bwd_multi(ctypes.addressof(_zproj_segs), len(segs), z.data_ptr(), dz.data_ptr(), B, d, Z,
                                   stream()), 'svae_zproj_bwd_multi')


def sumsq(g, n, part):
    check(lib.svae_sumsq(g.data_ptr(), n, part.data_ptr(), part.numel(), stream()), 'svae_sumsq')


def clip_grad(g, n, part, max_norm, norm_out=None):
    check(lib.svae_clip_grad(g.data_ptr(), n, part.data_ptr(), part.numel(), float(max_norm), ptr(norm_out), stream()),
          'svae_clip_grad')


def radam(p, pbf, g, m, v, n, part, scal, norm_out):
    check(lib.svae_radam(p.data_ptr(), ptr(pbf), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, part.data_ptr(),
                         part.numel(), scal.data_ptr(), ptr(norm_out), stream()), 'svae_radam')


# ---- fp32 kernel mode (argmax-reconstruction parity)
def gemm_f32(A, W, C, M, N_, K_, *, lda=None, ldw=None, ldc=None, epi=N.EPI_F32, bias=None, resid=None, ldr=0,
             rot=None, rot_cols=0, rot_d=0, rot_seq=0):
    _dev(A, W, C)
    check(lib.svae_gemm_f32(A.data_ptr(), W.data_ptr(), C.data_ptr(), M, N_, K_, lda or K_, ldw or K_, ldc or N_,
                            ptr(bias), ptr(resid), ldr, epi, ptr(rot), rot_cols, rot_d, rot_seq, stream()),
          'svae_gemm_f32')


def attention_f32(q, k, v, o, *, B, H, Lq, Lk, hd, sq, sk, sv, so, bq, bk, bv, bo, key_pad=None, causal=False,
                  window=0):
    check(lib.svae_attn_fwd_f32(q.data_ptr(), k.data_ptr(), v.data_ptr(), o.data_ptr(), sq, sk, sv, so, bq, bk, bv, bo,
                                ptr(key_pad), B, H, Lq, Lk, hd, int(causal), int(window), hd ** -0.5, stream()),
          'svae_attn_fwd_f32')


def layernorm_fwd_f32(x, w, b, y, rows, D):
    check(lib.svae_layernorm_fwd_f32(x.data_ptr(), w.data_ptr(), b.data_ptr(), y.data_ptr(), rows, D, stream()),
          'svae_layernorm_fwd_f32')


# ---- autoregressive decoding (f32; positions from the device scalar `cur`)
def dec_linear(X, W, Y, M, N_, K_, *, bias=None, resid=None, epi=N.EPI_F32, rot=None, rot_cols=0, rot_d=0, cur=None,
               ldx=None, ldw=None, ldy=None, ldr=None, part=None):
    """part: optional f32 workspace for split-K partials (the library splits narrow outputs when it fits)."""
    _dev(X, W, Y)
    assert X.dtype == f32 and W.dtype == f32 and Y.dtype == f32
    check(lib.svae_dec_linear(X.data_ptr(), ldx or K_, W.data_ptr(), ldw or K_, ptr(bias), Y.data_ptr(), ldy or N_,
                              ptr(resid), ldr or N_, M, N_, K_, epi, ptr(rot), rot_cols, rot_d, ptr(cur), ptr(part),
                              part.numel() if part is not None else 0, stream()), 'svae_dec_linear')


def dec_attn(qkv, kc, vc, O, B, H, hd, T, cur, window, scale=None, ldq=None, ldo=None):
    _dev(qkv, kc, vc, O, cur)
    check(lib.svae_dec_attn(qkv.data_ptr(), ldq or 3 * H * hd, kc.data_ptr(), vc.data_ptr(), B, H, hd, T,
                            cur.data_ptr(), window, hd ** -0.5 if scale is None else scale, O.data_ptr(),
                            ldo or H * hd, stream()), 'svae_dec_attn')


def dec_embed(out_ids, T, cur, table, x, B, D):
    assert out_ids.dtype == torch.int64
    check(lib.svae_dec_embed(out_ids.data_ptr(), T, cur.data_ptr(), table.data_ptr(), x.data_ptr(), B, D, stream()),
          'svae_dec_embed')


def dec_penalty(logits, rows, row_map, out_ids, T, cur, live, penalty):
    check(lib.svae_dec_penalty(logits.data_ptr(), logits.stride(0), rows, ptr(row_map), out_ids.data_ptr(), T,
                               cur.data_ptr(), ptr(live), penalty, stream()), 'svae_dec_penalty')


def dec_sample(logits, V, rows, row_map, out_ids, T, cur, live, end_token, temperature, top_k, top_p, seed,
               live_count=None):
    check(lib.svae_dec_sample(logits.data_ptr(), logits.stride(0), V, rows, ptr(row_map), out_ids.data_ptr(), T,
                              cur.data_ptr(), ptr(live), end_token, temperature, top_k, top_p,
                              seed & 0xFFFFFFFFFFFFFFFF, ptr(live_count), stream()), 'svae_dec_sample')


def dec_advance(cur):
    check(lib.svae_dec_advance(cur.data_ptr(), stream()), 'svae_dec_advance')
