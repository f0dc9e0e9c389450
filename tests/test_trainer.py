"""The fit loop (sparse_vae.Trainer) and the data-parallel batch sharding, on CPU with a stand-in model: the
micro-step / optimiser-step sequence under accumulate_grad_batches, the no_sync flag, epochs until max_steps,
validation scheduling, and equal disjoint per-rank shards (the condition for every rank to run the same number
of collectives)."""
import pytest
import torch

from sparse_vae import TextDataModule, Trainer
from sparse_vae.text_data_module import RankBatchSampler


class _Opt:
    def __init__(self, log):
        self.log = log

    def step(self):
        self.log.append('step')

    def zero_grad(self):
        self.log.append('zero')


class _Sched:
    def step(self):
        pass


class _Model:
    """Records what the Trainer calls, in order."""

    def __init__(self):
        self.log, self.logged, self.syncs, self.require_backward_grad_sync = [], {}, [], True
        self.w = torch.zeros(1, requires_grad=True)
        self.training = True

    def cuda(self):
        return self

    def initialize_weights(self):
        pass

    def setup(self, stage):
        pass

    def on_train_start(self):
        pass

    def train(self, mode=True):
        self.training = mode

    def configure_optimizers(self, tokens, accum):
        return [_Opt(self.log)], [{'scheduler': _Sched()}]

    def training_step(self, batch, i):
        self.syncs.append(self.require_backward_grad_sync)
        self.log.append('fwd')
        self.logged['train_nll'] = torch.tensor(1.0)
        return {'loss': (self.w * 1.0).sum()}

    def on_after_backward(self):
        self.log.append('oab')

    def validation_step(self, batch, i):
        self.logged['val_loss'] = torch.tensor(2.0 + i)


def _dm(n):
    return TextDataModule(dataset_name='synthetic', seq_len=8, batch_size=2, num_batches=n)


def test_accumulation_sequence_and_epochs():
    m = _Model()
    tr = Trainer(max_steps=5, accumulate_grad_batches=2, val_check_interval=None)
    tr.fit(m, datamodule=_dm(5))
    # epoch of 5 batches with accumulate 2: steps after micro-batches 2, 4 and 5 (epoch end); then epoch 2
    assert m.syncs[:5] == [False, True, False, True, True]
    assert m.syncs[5:] == [False, True, False, True]
    assert tr.global_step == 5 and m.log.count('step') == 5 and m.log.count('fwd') == 9
    assert m.require_backward_grad_sync is True


def test_validation_schedule():
    m = _Model()
    tr = Trainer(max_epochs=2, accumulate_grad_batches=1, val_check_interval=1.0, limit_val_batches=3)
    tr.fit(m, datamodule=_dm(4))
    assert len(tr.val_history) == 2                          # end of each epoch
    assert tr.val_history[0]['val_batches'] == 3
    assert tr.val_history[0]['val_loss'] == pytest.approx(3.0)   # mean of 2, 3, 4
    m = _Model()
    tr = Trainer(max_steps=6, val_check_interval=2, limit_val_batches=1)
    tr.fit(m, datamodule=_dm(100))
    assert [v['step'] for v in tr.val_history] == [2, 4, 6]


def test_rank_shards_are_disjoint_and_equal():
    dm = _dm(7)
    shards = [list(dm.train_dataloader(rank=r, world=3)) for r in range(3)]
    assert [len(s) for s in shards] == [2, 2, 2]              # 7 -> 6 batches: 2 per rank, tail dropped
    for r, s in enumerate(shards):
        for j, b in enumerate(s):
            want = dm.synthetic_batch(r + 3 * j)
            assert torch.equal(b['token_ids'].as_raw(), want['token_ids'].as_raw())


def test_rank_batch_sampler():
    class S:
        def __init__(self):
            self.b = [[i] for i in range(10)]

        def __len__(self):
            return len(self.b)

        def __iter__(self):
            return iter(self.b)

    got = [list(RankBatchSampler(S(), r, 4)) for r in range(4)]
    assert got == [[[0], [4]], [[1], [5]], [[2], [6]], [[3], [7]]]
    assert len(RankBatchSampler(S(), 0, 4)) == 2


def test_validation_keeps_training_logs_separate():
    """validation must not clear the training values logged before it, and its val_* keys must not
    leak into the next training log line."""
    class M(_Model):
        def validation_step(self, batch, i):
            self.logged.clear()
            self.logged['val_loss'] = torch.tensor(7.0)

    m = M()
    tr = Trainer(max_steps=4, val_check_interval=2, limit_val_batches=1, log_every_n_steps=1)
    tr.fit(m, datamodule=_dm(10))
    assert [v['val_loss'] for v in tr.val_history] == [7.0, 7.0]
    assert all('val_loss' not in h and 'train_nll' in h for h in tr.history)
    assert 'train_nll' in m.logged and 'val_loss' not in m.logged


def test_epoch_limit_defaults_like_lightning():
    assert Trainer().max_epochs == 1000
    assert Trainer(max_steps=10).max_epochs is None
    assert Trainer(max_epochs=3).max_epochs == 3
