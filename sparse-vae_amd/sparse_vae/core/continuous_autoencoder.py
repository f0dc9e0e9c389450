"""ContinuousVAE hparams and hooks (continuous_autoencoder.py:9-39 in the reference)."""
import math
from abc import ABC
from dataclasses import dataclass

import torch

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
    """on_train_start / KL annealing in on_after_backward (continuous_autoencoder.py:25-39), and the
    importance-weighted log-likelihood estimate used by test_step (continuous_autoencoder.py:55-88)."""

    @staticmethod
    def prior_log_prob(z):
        """continuous_autoencoder.py:55-57."""
        return -0.5 * z.pow(2.0).sum(dim=-1) - math.log(math.sqrt(2 * math.pi)) * z.shape[-1]

    @torch.no_grad()
    def estimate_log_prob_iw(self, q_of_z, x, labels, num_samples: int, num_iter: int = 1):
        """continuous_autoencoder.py:62-80. The num_iter chunks draw their z exactly as the reference does, but
        log p(x|z) of all num_samples draws is computed in one batched decoder pass (32K-token sub-batches),
        then combined chunk by chunk with the reference's own tensor shapes (so its [chunk, B, 1] + [chunk, B]
        broadcasting is reproduced)."""
        assert num_samples % num_iter == 0
        chunk_size = num_samples // num_iter
        zs = [q_of_z.rsample([chunk_size]) for _ in range(num_iter)]          # [chunk, B, 1, Z] each
        z_all = torch.cat(zs)
        S = z_all.shape[0]
        pad = getattr(x, 'padding', None)
        x = x.as_raw() if hasattr(x, 'as_raw') else x
        lpx_all = self.p_of_x_given_z(x.unsqueeze(0).expand(S, *x.shape), z_all,
                                      labels.expand(S, *labels.shape)[..., 1:], padding=pad)
        log_ws = []
        for it, z in enumerate(zs):
            log_p_of_z = self.prior_log_prob(z)                                # [chunk, B, 1]
            log_q_of_z = q_of_z.log_prob(z).sum(dim=-1)
            lpx = lpx_all[it * chunk_size:(it + 1) * chunk_size]                # [chunk, B]
            log_ws += [log_p_of_z + lpx - log_q_of_z]
        return torch.cat(log_ws).logsumexp(dim=0) - math.log(num_samples)

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
