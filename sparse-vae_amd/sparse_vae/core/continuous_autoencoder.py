"""ContinuousVAE hparams and hooks (continuous_autoencoder.py:9-39 in the reference)."""
from abc import ABC
from dataclasses import dataclass

from .language_model import LanguageModelHparams


@dataclass
class ContinuousVAEHparams(LanguageModelHparams, ABC):
    latent_depth: int = 64
    kl_annealing_steps: int = 0
    kl_weight_start: float = 1.0
    kl_weight_end: float = 1.0
    kl_weight: float = 1.0
    early_stopping_metric: str = 'val_loss'


class ContinuousVAEHooks:
    """on_train_start / KL annealing in on_after_backward (continuous_autoencoder.py:25-39)."""

    def on_train_start(self):
        self.hparams.kl_weight = self.hparams.kl_weight_start

    def anneal_kl(self):
        cur_step = self.global_step
        max_steps = self.hparams.kl_annealing_steps
        kl_end = self.hparams.kl_weight_end
        if not max_steps or self.hparams.kl_weight >= kl_end:
            return
        progress = cur_step / max_steps
        self.hparams.kl_weight = self.hparams.kl_weight_start + (kl_end - self.hparams.kl_weight_start) * progress
