"""marginal_kl (math_utils.py:51-58 in the reference): the train_mc_mutual_info diagnostic. Log-only (it
is not in the loss), so it runs as a handful of small device ops on [10, B, B, Z] tensors."""
import math

import torch


@torch.no_grad()
def marginal_kl(mu, scale, num_samples: int = 10, eps=None):
    eps = torch.randn((num_samples,) + tuple(mu.shape), device=mu.device) if eps is None else eps
    samples = mu + eps * scale
    x = samples[:, :, None]
    log_prob = -((x - mu) ** 2) / (2 * scale ** 2) - scale.log() - math.log(math.sqrt(2 * math.pi))
    cross = log_prob.sum(dim=-1)
    marginal = cross.logsumexp(dim=2) - math.log(samples.shape[1])
    sample_prob = -0.5 * (samples.pow(2.0).sum(dim=-1).mean() + samples.shape[-1] * math.log(2 * math.pi))
    return sample_prob - marginal.mean()
