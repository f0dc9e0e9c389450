"""Stub modules that let the UNMODIFIED reference (`/root/reference/sparse_vae`) import on CPU in the
survey container, for golden-vector generation only.

Seven modules are absent here: pytorch_lightning, omegaconf, torchtext, triton.ops.blocksparse, pynvml,
and the two reference modules the tree imports but does not ship (core/rotary_embedding.py,
core/activation_offload.py). Each stub is the minimal faithful form; none touches the dense hot path's
arithmetic, which runs entirely on stock PyTorch ATen CPU ops.
"""
import contextlib
import sys
import types

import torch
from torch import nn


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


class LightningModule(nn.Module):
    def __init__(self, *a, **k):
        super().__init__()
        self.logged = {}
        self.global_step = 0

    def save_hyperparameters(self, hp=None, *a, **k):
        import dataclasses
        if hp is None:
            return
        d = dataclasses.asdict(hp) if dataclasses.is_dataclass(hp) else dict(hp)
        object.__setattr__(self, '_hp', AttributeDict(d))

    @property
    def hparams(self):
        return self._hp

    @property
    def device(self):
        return torch.device('cpu')

    def log(self, name, value, *a, **k):
        self.logged[name] = value.detach().clone() if torch.is_tensor(value) else value


class _Anything:
    def __init__(self, *a, **k):
        pass


def install():
    def mod(name, **attrs):
        m = types.ModuleType(name)
        m.__dict__.update(attrs)
        sys.modules[name] = m
        return m

    pl = mod('pytorch_lightning', LightningModule=LightningModule, LightningDataModule=_Anything,
             Callback=_Anything, Trainer=_Anything, seed_everything=lambda s: torch.manual_seed(s))
    pl.callbacks = mod('pytorch_lightning.callbacks', EarlyStopping=_Anything,
                       LearningRateMonitor=_Anything, ModelCheckpoint=_Anything)
    pl.utilities = mod('pytorch_lightning.utilities')
    pl.utilities.parsing = mod('pytorch_lightning.utilities.parsing', AttributeDict=AttributeDict)
    pl.loggers = mod('pytorch_lightning.loggers', TensorBoardLogger=_Anything)
    pl.profiler = mod('pytorch_lightning.profiler', PyTorchProfiler=_Anything)
    mod('omegaconf', DictConfig=dict, OmegaConf=_Anything)
    tt = mod('torchtext')
    tt.data = mod('torchtext.data')
    tt.data.metrics = mod('torchtext.data.metrics', bleu_score=lambda *a, **k: 0.0)

    def _no_sparse(*a, **k):
        raise RuntimeError('triton.ops.blocksparse is not available; the dense path never calls it')

    import triton  # noqa: F401  (triton 3.6 is installed; only triton.ops is gone)
    mod('triton.ops')
    mod('triton.ops.blocksparse', matmul=_no_sparse, softmax=_no_sparse)
    mod('pynvml')

    class RotaryEmbedding:
        # Only used as a context manager whose consumer is commented out (attention.py:40).
        @staticmethod
        @contextlib.contextmanager
        def embedding_context(*a, **k):
            yield

    mod('sparse_vae.core.rotary_embedding', RotaryEmbedding=RotaryEmbedding)
    mod('sparse_vae.core.activation_offload', ActivationOffloadFunction=_Anything, offload=lambda *a, **k: None)


def import_reference(path='/root/reference'):
    import os
    os.environ.setdefault('PYTHONDONTWRITEBYTECODE', '1')
    sys.dont_write_bytecode = True
    install()
    if path not in sys.path:
        sys.path.insert(0, path)
    import sparse_vae  # noqa: F401
    return sys.modules['sparse_vae']
