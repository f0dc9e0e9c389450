"""Host logic: split-K counts of the paired weight-gradient launch (kernels.pair_splits): one round of <= 256
blocks, K-slices of similar length (>= 512 rows, whole 64-row K-tiles, none empty), a long-K GEMM split further than
its short-K partner."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = open(os.path.join(ROOT, 'sparse-vae_amd', 'sparse_vae', 'kernels.py')).read()
_ns = {'os': os}
exec(SRC[SRC.index('def pair_splits'):SRC.index('def linear_dw_pair')], _ns)   # the pure function (no GPU library)
pair_splits = _ns['pair_splits']


def _tiles(m, n):
    return -(-m // 256) * -(-n // 256)


def _check(shapes):
    sp = pair_splits(shapes)
    assert sp is not None
    blocks = sum(_tiles(m, n) * s for (m, n, _), s in zip(shapes, sp))
    assert blocks <= 256
    for (_, _, rows), s in zip(shapes, sp):
        kchunk = -(-(-(-rows // s)) // 64) * 64
        assert s >= 2 and kchunk >= 512 and (s - 1) * kchunk < rows      # no empty slice
    return sp, blocks


def test_pair_splits(monkeypatch):
    monkeypatch.delenv('SVAE_DW_PAIR_EQUAL', raising=False)
    sp, blocks = _check([(512, 512, 4096), (1024, 512, 32768)])        # C2 encoder: 96 -> ~250 blocks
    assert sp[1] > 4 * sp[0] and blocks >= 240
    assert _check([(512, 2048, 32768), (2048, 512, 32768)])[0] == (8, 8)   # C2 FFN pair unchanged
    sp, _ = _check([(768, 3072, 65536), (3072, 768, 65536)])              # C4 FFN pair: no extra slabs
    assert sp == (3, 3)
    sp, _ = _check([(768, 768, 4096), (1536, 768, 65536)])                # C4 encoder: the long GEMM split further
    assert sp[1] >= 12
    assert pair_splits([(512, 512, 512), (512, 512, 4096)]) is None       # a K too short to split
    monkeypatch.setenv('SVAE_DW_PAIR_EQUAL', '1')
    assert pair_splits([(512, 512, 4096), (1024, 512, 32768)]) == (8, 8)
