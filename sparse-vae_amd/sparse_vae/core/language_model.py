"""LanguageModel base (language_model.py:20-170 in the reference), without a hard Lightning dependency.

Keeps the hparams dataclass, `initialize_weights`, `get_nll`, `configure_optimizers` (RAdam + sqrt lr
scaling + cosine LambdaLR) and `on_after_backward` (clip + `grad_norm` log). If pytorch_lightning is
importable the class derives from LightningModule, so the reference's Trainer flow still works.
"""
import math
from abc import ABC
from dataclasses import dataclass, asdict, is_dataclass
from functools import partial
from typing import Optional

import torch
from torch import nn

try:  # optional: the image has no Lightning, the reference's train.py flow works if it is installed
    import pytorch_lightning as pl
    _Base = pl.LightningModule
except ImportError:  # pragma: no cover - the common case here
    pl = None
    _Base = nn.Module


class AttributeDict(dict):
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


@dataclass
class LanguageModelHparams(ABC):
    grad_clip_threshold: float = 5.0
    init_scale: Optional[float] = 0.02
    base_batch_size: int = 100_000
    lr: float = 2e-4
    lr_decay_steps: Optional[int] = 250_000
    start_token: Optional[int] = None
    end_token: Optional[int] = None
    early_stopping_metric: str = 'val_nll'
    log_samples: bool = True


def to_attrdict(hparams):
    if isinstance(hparams, AttributeDict):
        return hparams
    if is_dataclass(hparams):
        return AttributeDict(asdict(hparams))
    return AttributeDict(dict(hparams))


class LanguageModel(_Base, ABC):
    def __init__(self, hparams):
        super().__init__()
        object.__setattr__(self, '_hp', to_attrdict(hparams))
        self.start_token = self._hp.get('start_token')
        self.end_token = self._hp.get('end_token')
        self.logged = {}
        self._global_step = 0
        self.tokenizer = None

    # Lightning-compatible bits (used when Lightning is absent)
    @property
    def hparams(self):
        return self._hp

    @property
    def global_step(self):
        tr = getattr(self, '_trainer', None)
        return tr.global_step if tr is not None and hasattr(tr, 'global_step') else self._global_step

    def log(self, name, value, *args, **kwargs):
        self.logged[name] = value

    def setup(self, stage: Optional[str] = None):
        """language_model.py:57-66: take the datamodule's tokenizer and per-token byte counts (the class weights of
        the val_bpb metric, registered in half precision as in the reference) and the [CLS]/[SEP] ids."""
        tr = getattr(self, '_trainer', None)
        dm = getattr(tr, 'datamodule', None) if tr is not None else getattr(self, 'datamodule', None)
        if dm is None:
            return
        bpt = getattr(dm, 'bytes_per_token', None)
        if bpt is not None:
            self.token_weights = bpt.half()
        tok = getattr(dm, '_tokenizer', None)       # synthetic data has no tokenizer: [CLS]=1 / [SEP]=2 stay
        if tok is not None:
            self.tokenizer = tok
            if not self.start_token and not self.end_token:
                vocab = tok.get_vocab()
                self.start_token, self.end_token = vocab['[CLS]'], vocab['[SEP]']

    def initialize_weights(self):
        """language_model.py:80-96: N(0, init_scale) for Embedding/Linear weights, zero biases, LayerNorm
        untouched (learned queries keep their randn init)."""
        scale = self.hparams.init_scale
        if scale is None:
            return
        with torch.no_grad():
            for module in self.modules():
                if isinstance(module, (nn.BatchNorm1d, nn.LayerNorm)):
                    continue
                if isinstance(module, (nn.Embedding, nn.Linear)):
                    module.weight.normal_(0.0, scale)
                bias = getattr(module, 'bias', None)
                if isinstance(bias, torch.Tensor):
                    bias.zero_()

    def configure_optimizers(self, tokens_per_batch: int = None, accumulate_grad_batches: int = 1):
        """language_model.py:68-78: RAdam(lr * sqrt(tokens * accum / base_batch_size), wd 0.01) with a
        per-step cosine LambdaLR."""
        from .rectified_adam import RAdam
        if tokens_per_batch is None:
            tr = getattr(self, '_trainer', None)
            dm = getattr(tr, 'datamodule', None)
            tokens_per_batch = dm.hparams.tokens_per_batch if dm is not None else self.hparams.base_batch_size
            accumulate_grad_batches = getattr(tr, 'accumulate_grad_batches', accumulate_grad_batches)
        lr_scale = (tokens_per_batch * accumulate_grad_batches / self.hparams.base_batch_size) ** 0.5
        opt = RAdam(self, lr=self.hparams.lr * lr_scale, weight_decay=0.01)
        sched = torch.optim.lr_scheduler.LambdaLR(opt, partial(cosine_decay, self.hparams.lr_decay_steps))
        return [opt], [{'scheduler': sched, 'interval': 'step'}]

    def on_after_backward(self):
        """language_model.py:120-122: the global grad norm is computed here (and logged); the clip itself is
        fused into the RAdam kernel, which reads the same norm on the device."""
        norm = self.grad_norm()
        self.log('grad_norm', norm)

    def sample(self, max_length: int, batch_size: int = 1, **kwargs):
        return None


def cosine_decay(decay_steps: int, cur_step: int):
    """language_model.py:135-141."""
    progress = cur_step / max(1, decay_steps)
    if progress >= 1.0:
        print('Learning rate decayed to 0.0. Halting training.')
        raise KeyboardInterrupt
    return max(0.0, 0.5 * (1.0 + math.cos(math.pi * progress)))
