"""Host logic: the vocabulary head's dW split-K choice (engine._head_dw_splits) fills the last wave of 256 x 256
tiles: C2 (V 32768, d 512: 256 tiles) one split, C4 / C5 (d 768: 384 tiles on 256 CUs) two."""
import os
import sys
import types

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))


def test_head_dw_splits(monkeypatch):
    from sparse_vae.engine import VAEEngine
    monkeypatch.delenv('SVAE_HEAD_DW_SPLITS', raising=False)
    eng = types.SimpleNamespace(ncu=256)
    f = VAEEngine._head_dw_splits
    assert f(eng, 32768, 512) == 1          # C2
    assert f(eng, 32768, 768) == 2          # C4, C5
    assert f(eng, 32768, 1024) == 1         # 512 tiles: two full waves
    assert f(eng, 1024, 256) == 1           # small models: fewer tiles than CUs, unchanged
    monkeypatch.setenv('SVAE_HEAD_DW_SPLITS', '3')
    assert f(eng, 32768, 512) == 3
