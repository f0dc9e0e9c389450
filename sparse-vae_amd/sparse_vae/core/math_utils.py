"""marginal_kl (math_utils.py:51-58 in the reference): the Monte-Carlo marginal KL behind the train_mc_mutual_info
diagnostic, on the fused HIP kernel pair (`svae_mutual_info`: mi_marginal + mi_final) the training step uses
through engine.mutual_info. Same signature as the reference (a Normal posterior [B, 1, Z], num_samples draws);
`eps` [num_samples, B, Z] injects the N(0, 1) draws (parity tests), otherwise they are drawn in-kernel from a seed
taken from torch's generator. No CPU fallback."""
import torch

from .. import kernels as K


@torch.no_grad()
def marginal_kl(posteriors, num_samples: int = 10, eps=None):
    mu, scale = posteriors.loc, posteriors.scale
    if not mu.is_cuda:
        raise RuntimeError('marginal_kl runs on the MI355X HIP kernels (svae_mutual_info): no CPU fallback')
    B, Z = mu.shape[0], mu.shape[-1]
    if mu.numel() != B * Z:
        raise ValueError('marginal_kl expects a posterior of shape [B, 1, latent] (transformer_vae.py:52-61)')
    # the kernel's posterior statistics row: mu | logvar (scale = exp(logvar / 2))
    stats = torch.cat([mu.reshape(B, Z).float(), 2.0 * scale.reshape(B, Z).float().log()], dim=1).contiguous()
    zero = torch.zeros(1, dtype=torch.float32, device=mu.device)
    out = torch.empty((), dtype=torch.float32, device=mu.device)
    ws = torch.empty(2 * num_samples * B, dtype=torch.float32, device=mu.device)
    if eps is not None:
        eps = eps.to(mu.device, torch.float32).reshape(num_samples, B, Z).contiguous()
    seed = int(torch.randint(0, 2 ** 62, (1,)).item())
    K.mutual_info(stats, zero, B, Z, seed, out, ws, eps=eps, S=num_samples)   # out = 0 - marginal_kl
    return -out
