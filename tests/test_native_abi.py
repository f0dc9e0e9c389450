"""The C-ABI library loads and exports every entry point declared in include/svae.h (no compute calls:
this runs on CPU). Also checks the ctypes descriptor layouts against the header's field order."""
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, 'include', 'svae.h')


def header_functions():
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    return sorted(set(re.findall(r'^\s*(?:int|int32_t|int64_t|const char\*)\s+(svae_\w+)\s*\(', src, flags=re.M)))


def header_struct_fields(name):
    src = open(HEADER).read()
    src = re.sub(r'/\*.*?\*/', '', src, flags=re.S)
    body = re.search(r'typedef struct %s \{(.*?)\} %s;' % (name, name), src, flags=re.S).group(1)
    fields = []
    for decl in body.split(';'):
        decl = decl.strip()
        if not decl:
            continue
        decl = re.sub(r'^(const\s+)?\w+\s*\**', '', decl)
        fields += [f.strip().lstrip('*') for f in decl.split(',')]
    return fields


def test_library_exports_every_header_symbol():
    from sparse_vae import _native
    names = header_functions()
    assert len(names) >= 20
    for n in names:
        assert hasattr(_native.lib, n), n
    assert set(names) == set(_native.EXPORTED)


def test_version_string():
    from sparse_vae import _native
    assert _native.lib.svae_version().startswith(b'libsvae')


@pytest.mark.parametrize('struct,cls', [('svae_gemm_desc', 'GemmDesc'), ('svae_attn_desc', 'AttnDesc')])
def test_ctypes_layout_matches_header(struct, cls):
    from sparse_vae import _native
    got = [f[0] for f in getattr(_native, cls)._fields_]
    assert got == header_struct_fields(struct)


def test_bad_arguments_are_rejected_without_launch():
    """Argument validation happens before any launch, so it is testable without a GPU."""
    import ctypes
    from sparse_vae import _native
    d = _native.GemmDesc()
    assert _native.lib.svae_gemm(ctypes.byref(d), None) == 1          # NULL operands
    d.A, d.B, d.C = 16, 16, 16
    d.M, d.N, d.K, d.batch, d.splits = 128, 128, 60, 1, 1            # K % 8 != 0
    d.lda, d.ldb, d.ldc = 64, 64, 128
    assert _native.lib.svae_gemm(ctypes.byref(d), None) == 1
    assert _native.lib.svae_layernorm_fwd(None, 0, None, None, None, None, None, 4, 64, None) == 1
    a = _native.AttnDesc()
    assert _native.lib.svae_attn_fwd(ctypes.byref(a), None) == 1


def test_product_refuses_cpu_execution():
    """No CPU fallback: the model builds on CPU (state_dict, hparams) but the step refuses to run there."""
    import torch
    from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule
    m = TransformerVAE(TransformerVAEHparams(d_model=128, num_layers=4, num_heads=8, sparse_self_attention=False),
                       device='cpu')
    batch = TextDataModule(dataset_name='synthetic', seq_len=128, batch_size=2).synthetic_batch(0)
    with pytest.raises(RuntimeError, match='no CPU fallback|There is no CPU fallback'):
        m.training_step(batch, 0)


def test_colsum_seg_layout():
    """svae_colsum_seg: the ctypes mirror matches the header (field order and size)."""
    import ctypes
    from sparse_vae import _native as N
    assert ctypes.sizeof(N.ColsumSeg) == 32
    assert [f[0] for f in N.ColsumSeg._fields_] == ['inp', 'out', 'ld', 'rows', 'cols']
    hdr = open(os.path.join(ROOT, 'include', 'svae.h')).read()
    assert '#define SVAE_COLSUM_MAX 8' in hdr and N.COLSUM_MAX == 8


def test_zproj_seg_layout():
    """svae_zproj_seg: the ctypes mirror matches the header (four pointers, 32 B) and the segment cap."""
    import ctypes
    from sparse_vae import _native as N
    assert ctypes.sizeof(N.ZprojSeg) == 32
    assert [f[0] for f in N.ZprojSeg._fields_] == ['g', 'W', 'dW', 'db']
    hdr = open(os.path.join(ROOT, 'include', 'svae.h')).read()
    assert '#define SVAE_ZPROJ_MAX 32' in hdr and N.ZPROJ_MAX == 32


def test_zproj_fwd_seg_layout():
    """svae_zproj_fwd_seg: three pointers, 24 B, in header order."""
    import ctypes
    from sparse_vae import _native as N
    assert ctypes.sizeof(N.ZprojFwdSeg) == 24
    assert [f[0] for f in N.ZprojFwdSeg._fields_] == ['W', 'bias', 'out']
