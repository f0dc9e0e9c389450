"""ctypes binding of libsvae.so (the C ABI declared in include/svae.h).

There is deliberately no fallback: if the HIP library is missing or fails to load, importing the model
raises. Every wrapper validates shapes/dtypes/devices on the host before the call and raises
RuntimeError on a non-zero status.
"""
import ctypes
import os

import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('SVAE_LIB') or os.path.join(_HERE, 'libsvae.so')   # SVAE_LIB: A/B builds

c_void_p, c_int32, c_int64, c_float, c_uint64 = (ctypes.c_void_p, ctypes.c_int32, ctypes.c_int64,
                                                  ctypes.c_float, ctypes.c_uint64)
c_fptr = ctypes.c_void_p

EPI_BF16, EPI_F32, EPI_F32_ACC, EPI_F32_ATOMIC, EPI_GELU, EPI_GELU_BWD, EPI_DROPOUT_RESID, \
    EPI_ROTARY_BF16, EPI_CE_STATS, EPI_CE_PROB, EPI_ROWSCALE_GATHER = range(11)


class GemmDesc(ctypes.Structure):
    _fields_ = [
        ('A', c_void_p), ('B', c_void_p),
        ('lda', c_int64), ('ldb', c_int64), ('batch_stride_a', c_int64), ('batch_stride_b', c_int64),
        ('M', c_int32), ('N', c_int32), ('K', c_int32),
        ('batch', c_int32), ('splits', c_int32),
        ('a_t', c_int32), ('b_t', c_int32),
        ('epi', c_int32),
        ('C', c_void_p),
        ('ldc', c_int64), ('batch_stride_c', c_int64),
        ('bias', c_void_p), ('resid', c_void_p), ('ldr', c_int64),
        ('aux', c_void_p), ('ldaux', c_int64),
        ('alpha', c_float), ('drop_p', c_float), ('seed', c_uint64),
        ('rot_tab', c_void_p), ('rot_cols', c_int32), ('rot_d', c_int32), ('rot_seq', c_int32),
        ('labels', c_void_p), ('label_logit', c_void_p),
        ('a_rowsum', c_void_p),
        ('k_weight', c_void_p), ('row_a', c_void_p), ('row_b', c_void_p), ('gather', c_void_p), ('ldg', c_int64),
        ('delta', c_void_p), ('delta_o32', c_void_p), ('ld_o32', c_int64), ('delta_hd', c_int32), ('delta_seq', c_int32),
    ]


class AttnDesc(ctypes.Structure):
    _fields_ = [
        ('q', c_void_p), ('k', c_void_p), ('v', c_void_p), ('o', c_void_p),
        ('sq', c_int64), ('sk', c_int64), ('sv', c_int64), ('so', c_int64),
        ('bq', c_int64), ('bk', c_int64), ('bv', c_int64), ('bo', c_int64),
        ('key_pad', c_void_p), ('lse', c_void_p),
        ('B', c_int32), ('H', c_int32), ('Lq', c_int32), ('Lk', c_int32), ('hd', c_int32), ('causal', c_int32),
        ('scale', c_float),
        ('dout', c_void_p), ('sdo', c_int64), ('bdo', c_int64),
        ('delta', c_void_p), ('dq', c_void_p), ('bdq', c_int64),
        ('dk', c_void_p), ('dv', c_void_p),
        ('sdk', c_int64), ('sdv', c_int64), ('bdk', c_int64), ('bdv', c_int64),
        ('rot_tab', c_void_p), ('rot_d', c_int32),
        ('o32', c_void_p), ('so32', c_int64), ('bo32', c_int64),
        ('dq_part', c_void_p), ('dq_bf', c_void_p), ('ldq_bf', c_int64),
        ('window', c_int32),
        ('delta_ready', c_int32),
        ('o_lo', c_void_p), ('so_lo', c_int64), ('bo_lo', c_int64),
        ('fwd_ws', c_void_p), ('fwd_ws_elems', c_int64),
    ]


COLSUM_MAX = 8
LN_MULTI_MAX = 4        # SVAE_LN_MULTI_MAX


ZPROJ_MAX = 32


class ZprojSeg(ctypes.Structure):
    """svae_zproj_seg (include/svae.h)."""
    _fields_ = [('g', c_void_p), ('W', c_void_p), ('dW', c_void_p), ('db', c_void_p)]


class ZprojFwdSeg(ctypes.Structure):
    """svae_zproj_fwd_seg (include/svae.h)."""
    _fields_ = [('W', c_void_p), ('bias', c_void_p), ('out', c_void_p)]


class ColsumSeg(ctypes.Structure):
    """svae_colsum_seg (include/svae.h)."""
    _fields_ = [('inp', c_void_p), ('out', c_void_p), ('ld', c_int64), ('rows', c_int32), ('cols', c_int32)]


_SIGS = {
    'svae_gemm': [ctypes.POINTER(GemmDesc), c_void_p],
    'svae_gemm_pair': [ctypes.POINTER(GemmDesc), ctypes.POINTER(GemmDesc), c_void_p],
    'svae_resid_ln_fwd': [c_void_p, c_void_p, c_int32, c_int64, c_float, c_uint64, c_void_p, c_int32, c_void_p,
                          c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_layernorm_fwd': [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                           c_void_p],
    'svae_layernorm_bwd': [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                           c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p],
    'svae_layernorm_bwd_drop': [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_float, c_uint64, c_int32,
                                c_void_p, c_void_p, c_void_p],
    'svae_layernorm_bwd_gelu': [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                c_void_p, c_int32, c_int32, c_int32, c_void_p],
    'svae_layernorm_nblk': [c_int32],
    'svae_colsum': [c_void_p, c_int32, c_int32, c_int32, c_int64, c_void_p, c_int32, c_void_p],
    'svae_colsum_multi': [c_void_p, c_int32, c_void_p],
    'svae_attn_fwd': [ctypes.POINTER(AttnDesc), c_void_p],
    'svae_attn_bwd': [ctypes.POINTER(AttnDesc), c_void_p],
    'svae_attn_dq_part_elems': [c_int32, c_int32, c_int32, c_int32, c_int32],
    'svae_attn_dq_part_elems_w': [c_int32, c_int32, c_int32, c_int32, c_int32, c_int32],
    'svae_attn_fwd_ws_elems': [c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32],
    'svae_transpose_blocks': [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_dq_finalize': [c_void_p, c_void_p, c_int64, c_int32, c_int32, c_void_p, c_int32, c_void_p],
    'svae_embedding_fwd': [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_embedding_fwd_dual': [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_embedding_bwd': [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_reparam_kl_fwd': [c_void_p, c_void_p, c_uint64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                            c_void_p, c_int32, c_int32, c_void_p],
    'svae_reparam_kl_bwd': [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_ce_finalize': [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p,
                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    'svae_ce_weighted_nll': [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                             c_void_p],
    'svae_ce_red_ws_elems': [c_int32],
    'svae_clip_grad': [c_void_p, c_int64, c_void_p, c_int32, c_float, c_void_p, c_void_p],
    'svae_ce_label_logit': [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_int32, c_void_p,
                            c_void_p],
    'svae_ce_prob_finalize': [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p,
                              c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    'svae_ce_prob_finalize_fix': [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p,
                                  c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_void_p,
                                  c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p],
    'svae_ce_prob_bwd_prep': [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32,
                              c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p],
    'svae_embedding_bwd_ce': [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p],
    'svae_ce_grad': [c_void_p, c_int64, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32,
                     c_int32, c_int32, c_void_p],
    'svae_dropout_bwd_cast': [c_void_p, c_void_p, c_float, c_uint64, c_int64, c_int32, c_int64, c_void_p],
    'svae_gelu_bwd': [c_void_p, c_void_p, c_void_p, c_int64, c_void_p],
    'svae_prep_tokens': [c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p, c_void_p, c_void_p,
                         c_void_p, c_void_p],
    'svae_step_scalars': [c_void_p, c_void_p, c_void_p, c_float, c_void_p, c_void_p, c_void_p],
    'svae_zproj_bwd_multi': [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    'svae_zproj_fwd_multi': [c_void_p, c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    'svae_layernorm_fwd_multi': [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32,
                                 c_void_p],
    'svae_layernorm_bwd_multi': [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                 c_int32, c_int32, c_int32, c_int32, c_void_p],
    'svae_layernorm_fwd_z': [c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32,
                             c_int32, c_void_p],
    'svae_cast_bf16': [c_void_p, c_void_p, c_int64, c_void_p],
    'svae_extract_rows': [c_void_p, c_int64, c_int32, c_int32, c_int32, c_void_p, c_void_p],
    'svae_zproj_bwd': [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    'svae_sumsq': [c_void_p, c_int64, c_void_p, c_int32, c_void_p],
    'svae_radam': [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_void_p, c_int32, c_void_p,
                   c_void_p, c_void_p],
    'svae_gemm_f32': [c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int64, c_int64, c_int64, c_void_p,
                      c_void_p, c_int64, c_int32, c_void_p, c_int32, c_int32, c_int32, c_void_p],
    'svae_attn_fwd_f32': [c_void_p, c_void_p, c_void_p, c_void_p, c_int64, c_int64, c_int64, c_int64, c_int64, c_int64,
                          c_int64, c_int64, c_void_p, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32, c_int32,
                          c_float, c_void_p],
    'svae_layernorm_fwd_f32': [c_void_p, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_ce_seq_logprob': [c_void_p, c_int32, c_void_p, c_void_p, c_int32, c_int32, c_void_p, c_void_p],
    'svae_dec_linear': [c_void_p, c_int64, c_void_p, c_int64, c_void_p, c_void_p, c_int64, c_void_p, c_int64, c_int32,
                        c_int32, c_int32, c_int32, c_void_p, c_int32, c_int32, c_void_p, c_void_p, c_int64, c_void_p],
    'svae_dec_attn': [c_void_p, c_int64, c_void_p, c_void_p, c_int32, c_int32, c_int32, c_int32, c_void_p, c_int32,
                      c_float, c_void_p, c_int64, c_void_p],
    'svae_dec_embed': [c_void_p, c_int32, c_void_p, c_void_p, c_void_p, c_int32, c_int32, c_void_p],
    'svae_dec_penalty': [c_void_p, c_int64, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_float,
                         c_void_p],
    'svae_dec_sample': [c_void_p, c_int64, c_int32, c_int32, c_void_p, c_void_p, c_int32, c_void_p, c_void_p, c_int32,
                        c_float, c_int32, c_float, c_uint64, c_void_p, c_void_p],
    'svae_dec_advance': [c_void_p, c_void_p],
    'svae_mutual_info': [c_void_p, c_void_p, c_uint64, c_void_p, c_int32, c_int32, c_int32, c_void_p, c_void_p,
                         c_void_p],
    'svae_version': [],
}


def _load():
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f'libsvae.so not found at {LIB_PATH}: build it with `make -C sparse-vae_amd` '
                           f'(or __graft_entry__.build()). There is no CPU fallback.')
    lib = ctypes.CDLL(LIB_PATH)
    for name, argtypes in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = argtypes
        fn.restype = {'svae_version': ctypes.c_char_p, 'svae_attn_dq_part_elems': c_int64,
                      'svae_attn_dq_part_elems_w': c_int64, 'svae_attn_fwd_ws_elems': c_int64}.get(name, ctypes.c_int)
    return lib


lib = _load()
EXPORTED = tuple(_SIGS)


def check(status, name):
    if status != 0:
        raise RuntimeError(f'{name} failed with status {status}')


def ptr(t):
    return None if t is None else t.data_ptr()


def stream():
    return torch.cuda.current_stream().cuda_stream
