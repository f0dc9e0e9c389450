"""The drop-in CLI end to end on the device: `python train.py transformer-vae preset=tiny ...` (reference
train.py:12-95) run in-process through sparse_vae.Trainer -- synthetic TextDataModule batches, RAdam + cosine
LambdaLR, the logged keys of the reference's training_step / on_after_backward, validation (val_loss, val_bpb),
and gradient accumulation (the reference's default accumulate_grad_batches=2, train.py:16-23)."""
import math
import os

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, tmp_path, monkeypatch):
    import sys
    sys.path.insert(0, ROOT)
    import train
    monkeypatch.chdir(tmp_path)
    return train.main(['train.py', 'transformer-vae'] + args)


def test_train_py_preset_tiny(tmp_path, monkeypatch):
    tr = _run(['preset=tiny', 'trainer.max_steps=3', 'trainer.log_every_n_steps=1', 'trainer.val_check_interval=2',
               'trainer.limit_val_batches=2'], tmp_path, monkeypatch)
    assert tr.global_step == 3 and len(tr.history) == 3
    for logs in tr.history:
        for k in ('train_kl', 'train_nll', 'train_mc_mutual_info', 'grad_norm'):
            assert k in logs and math.isfinite(logs[k]), (k, logs)
        assert 9.0 < logs['train_nll'] < 11.5          # ~ln(32768) at init
        assert logs['grad_norm'] > 0
    assert [v['step'] for v in tr.val_history] == [2]
    v = tr.val_history[0]
    assert v['val_batches'] == 2 and math.isfinite(v['val_loss']) and math.isfinite(v['val_bpb'])
    # synthetic data: one byte per token, unit class weights -> val_bpb = val_nll / ln 2
    assert abs(v['val_bpb'] - v['val_nll'] / math.log(2)) < 1e-3 * v['val_bpb']
    m, opt = tr.model, tr.optimizer
    assert opt.param_groups[0]['step'] == 4
    assert opt.exp_avg.abs().sum().item() > 0
    # initialize_weights zeroed every bias; three RAdam steps moved them
    assert m.q_of_z_given_x.linear.bias.abs().sum().item() > 0
    assert torch.isfinite(m._flat.master).all()


def test_accumulation_matches_one_big_batch(tmp_path):
    """accumulate_grad_batches=2 over two half batches applies the same update as one step on the whole batch
    (loss / 2 per micro-step, the first micro-gradient clipped in place only when over the threshold)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, 'sparse-vae_amd'))
    from sparse_vae import TransformerVAE, TransformerVAEHparams, TextDataModule

    def model():
        torch.manual_seed(5)
        hp = TransformerVAEHparams(d_model=128, num_layers=4, num_heads=8, sparse_self_attention=False,
                                   grad_clip_threshold=1e6)
        m = TransformerVAE(hp, device='cuda')
        m.initialize_weights()
        return m

    dm = TextDataModule(dataset_name='synthetic', seq_len=128, batch_size=8)
    full = dm.synthetic_batch(0, device='cuda')
    ids = full['token_ids'].as_raw()
    eps = torch.randn(8, 1, 64, device='cuda')
    halves = [{'token_ids': ids[h * 4:(h + 1) * 4], 'num_tokens': full['num_tokens'][h * 4:(h + 1) * 4],
               'num_bytes': full['num_bytes'][h * 4:(h + 1) * 4]} for h in range(2)]
    a, b = model(), model()
    # a: two micro-steps of 4 sequences (loss / 2 each)
    for h, sync in ((0, False), (1, True)):
        a.require_backward_grad_sync = sync
        out = a.training_step(halves[h], h, eps=eps[h * 4:(h + 1) * 4], dropout=0.0)
        (out['loss'] / 2).backward()
        a.on_after_backward()
    # b: one step on all 8 (same per-sequence token counts -> the mean of the two half-batch means)
    out = b.training_step(full, 0, eps=eps, dropout=0.0)
    out['loss'].backward()
    b.on_after_backward()
    ga, gb = a._flat.grad[:a._flat.n_live].double(), b._flat.grad[:b._flat.n_live].double()
    # equal in exact arithmetic; the two runs differ by bf16 rounding (different GEMM row blocks): ~1 % of the
    # norm. A scaling bug (a micro-gradient dropped, doubled or left unhalved) moves the norm by >= 25 %.
    cos = (ga @ gb / (ga.norm() * gb.norm())).item()
    assert cos > 0.999 and abs(ga.norm().item() / gb.norm().item() - 1) < 0.01, (cos, ga.norm(), gb.norm())
