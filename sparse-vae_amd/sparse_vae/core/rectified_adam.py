"""RAdam (rectified_adam.py:6-88 in the reference), fused over the flat parameter arena.

One `svae_sumsq` + one `svae_radam` launch per step replace the per-parameter loop: the kernel reads the
global grad norm, applies the clip of `on_after_backward` (language_model.py:120-122), updates m, v and
the f32 master weights, and writes the bf16 shadow the GEMMs read. Step-dependent scalars (rectification
term r_t, bias corrections, LambdaLR-scheduled lr) are computed on the host exactly as the reference does
and handed to the device through a ring of pinned buffers (no host sync).
"""
import torch
from torch.optim import Optimizer

from .. import kernels as K


class RAdam(Optimizer):
    def __init__(self, model, lr=1e-3, betas=(0.9, 0.999), eps=1e-6, weight_decay=1e-6, lamb=False,
                 max_grad_norm=None):
        assert 0.0 <= lr and 0.0 <= eps and 0.0 <= betas[0] < 1.0 and 0.0 <= betas[1] < 1.0 and 0.0 <= weight_decay
        if lamb:
            raise NotImplementedError('LAMB variant (rectified_adam.py:73-80) is unused by the reference')
        self.model = model
        self.flat = model._flat
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay, lamb=lamb)
        super().__init__([p for p in model.parameters()], defaults)
        self.max_grad_norm = (max_grad_norm if max_grad_norm is not None
                              else float(model.hparams.get('grad_clip_threshold', 5.0)))
        dev = self.flat.device
        n = self.flat.n_live
        self.exp_avg = torch.zeros(n, device=dev)
        self.exp_avg_sq = torch.zeros(n, device=dev)
        self._scal_dev = torch.zeros(9, device=dev)
        self._ring = [torch.zeros(9).pin_memory() for _ in range(4)]
        self._ring_ev = [None] * 4
        self._ring_i = 0
        self.norm_out = torch.zeros(1, device=dev)

    def step_scalars(self, group):
        """The host arithmetic of rectified_adam.py:26-37, 82."""
        beta1, beta2 = group['betas']
        lr = group['lr']
        step = group.setdefault('step', 1)
        beta2_t = beta2 ** step
        bcv = (1 - beta2_t) ** 0.5
        rho_inf = 2.0 / (1.0 - beta2) - 1.0
        rho_t = rho_inf - 2 * step * beta2_t / (1 - beta2_t)
        if rho_t > 4:
            r_t = (((rho_t - 4.0) * (rho_t - 2.0) * rho_inf) / ((rho_inf - 4.0) * (rho_inf - 2.0) * rho_t)) ** 0.5
            lr *= r_t * bcv
        bcm = 1 - beta1 ** step
        return [lr, bcm, bcv, float(rho_t > 4), beta1, beta2, group['eps'], group['weight_decay'], self.max_grad_norm]

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        group = self.param_groups[0]
        i = self._ring_i
        if self._ring_ev[i] is not None:
            self._ring_ev[i].synchronize()
        self._ring[i].copy_(torch.tensor(self.step_scalars(group)))
        self._scal_dev.copy_(self._ring[i], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._ring_ev[i] = ev
        self._ring_i = (i + 1) % len(self._ring)
        flat = self.flat
        n = flat.n_live
        part = self.model._norm_partials(fresh=False)
        K.radam(flat.master, flat.shadow, flat.grad, self.exp_avg, self.exp_avg_sq, n, part, self._scal_dev,
                self.norm_out)
        flat.refresh_transposed()                    # dX GEMMs read W^T copies of the shadow
        flat.shadow_version = flat.master._version   # the kernel kept the bf16 shadow in sync
        self.model._norm_valid = False
        group['step'] += 1
        return loss

    def zero_grad(self, set_to_none: bool = False):
        self.model.zero_grad_flat()
