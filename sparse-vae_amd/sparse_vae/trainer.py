"""A minimal Trainer for the reference's fit loop (pytorch_lightning is not installed here).

Mirrors what Lightning does for the reference (train.py:12-95 builds `Trainer(**config.trainer)` and calls
`fit(model, datamodule)`):

* epochs over the train dataloader until `max_steps` optimiser steps (or `max_epochs`) -- the reference's
  cosine schedule ends training by raising KeyboardInterrupt (language_model.py:135-141);
* per micro-batch: training_step -> (loss / accumulate_grad_batches).backward() -> on_after_backward; every
  `accumulate_grad_batches` micro-batches (and at the end of an epoch) RAdam.step (fused clip + update) ->
  LambdaLR.step -> zero_grad. `model.require_backward_grad_sync` is False on the micro-steps no optimiser step
  follows (DDP's no_sync): their backward all-reduces nothing;
* validation (`validation_step` over the val loader, logged values averaged over its batches) every
  `val_check_interval` training batches (int), or that fraction of an epoch (float; 1.0 = end of each epoch),
  `limit_val_batches` batches at most.

Data parallel: one process per GPU (torch.distributed.run); RANK/LOCAL_RANK/WORLD_SIZE come from the
environment and the backend is 'nccl' (RCCL on ROCm). The datamodule hands each rank a disjoint shard of the
batches with the same batch count on every rank (the tail that does not divide by the world size is dropped,
as DistributedSampler(drop_last=True) does), so every rank runs the same number of collectives.
"""
import os
import time

import torch
import torch.distributed as dist


def seed_everything(seed: int):
    import random
    import numpy as np
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    return seed


def init_distributed():
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if torch.cuda.is_available():
        torch.cuda.set_device(local)
    if world > 1 and not dist.is_initialized():
        dist.init_process_group('nccl' if torch.cuda.is_available() else 'gloo')
    return world, (dist.get_rank() if world > 1 else 0), local


def _scalar(v):
    return v.item() if torch.is_tensor(v) else v


class Trainer:
    def __init__(self, max_steps: int = -1, max_epochs=None, accumulate_grad_batches: int = 1,
                 log_every_n_steps: int = 50, val_check_interval=1.0, limit_val_batches=None, gpus=None,
                 precision='bf16', **unused):
        self.max_steps = max_steps
        # Lightning's default: 1000 epochs when neither limit is set (the cosine schedule's KeyboardInterrupt
        # usually ends training first)
        self.max_epochs = 1000 if max_epochs is None and (max_steps is None or max_steps <= 0) else max_epochs
        self.accumulate_grad_batches = max(1, int(accumulate_grad_batches))
        self.log_every_n_steps = log_every_n_steps
        self.val_check_interval = val_check_interval
        self.limit_val_batches = limit_val_batches
        self.global_step = 0
        self.current_epoch = 0
        self.datamodule = None
        self.history = []
        self.val_history = []
        self.rank = 0

    # ------------------------------------------------------------------ loop pieces
    def _val_every(self, loader):
        """Training batches between validation runs (None: end of epoch only)."""
        v = self.val_check_interval
        if v is None:
            return None
        if isinstance(v, int) and not isinstance(v, bool) and v >= 1:
            return v
        n = len(loader) if hasattr(loader, '__len__') else None
        if n is None or float(v) >= 1.0:
            return None
        return max(1, int(n * float(v)))

    @torch.no_grad()
    def validate(self, model):
        """Mean of the val_* values over the validation batches (and, under data parallelism, over the ranks'
        batches). The training values logged before it are restored afterwards, so the next training log line
        carries no val_* key."""
        dm = self.datamodule
        saved = dict(model.logged)
        sums, counts, count = {}, {}, 0
        try:
            for j, batch in enumerate(dm.val_dataloader()):
                if self.limit_val_batches is not None and j >= int(self.limit_val_batches):
                    break
                model.logged.clear()
                model.validation_step(batch, j)
                for k, v in model.logged.items():
                    if k.startswith('val_'):
                        sums[k] = sums.get(k, 0.0) + float(_scalar(v))
                        counts[k] = counts.get(k, 0) + 1
                count += 1
        finally:
            model.logged.clear()
            model.logged.update(saved)
        if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
            # the ranks may hold different key sets (`val_mc_mutual_info` only where some batch had > 1 sequence):
            # agree on the union of the names first, then reduce one fixed-length vector of per-key sums and
            # per-key batch counts (0 where this rank has no value)
            names = [None] * dist.get_world_size()
            dist.all_gather_object(names, sorted(sums))
            keys = sorted(set().union(*names))
            t = torch.tensor([sums.get(k, 0.0) for k in keys] + [float(counts.get(k, 0)) for k in keys]
                             + [float(count)], dtype=torch.float64,
                             device=model.device if dist.get_backend() == 'nccl' else 'cpu')
            dist.all_reduce(t)
            n = len(keys)
            sums = {k: float(t[i]) for i, k in enumerate(keys)}
            counts = {k: int(round(float(t[n + i]))) for i, k in enumerate(keys)}
            count = int(round(float(t[-1])))
        # each key is the mean over the batches that logged it (Lightning's epoch-level mean of a logged value)
        logs = {k: v / max(counts.get(k, 0), 1) for k, v in sums.items()}
        logs['step'] = self.global_step
        logs['val_batches'] = count
        self.val_history.append(logs)
        if self.rank == 0:
            print(logs, flush=True)
        return logs

    def fit(self, model, datamodule=None):
        world, rank, local = init_distributed()
        self.rank = rank
        self.datamodule = datamodule
        model._trainer = self
        if torch.cuda.is_available():
            model.cuda()
        model.initialize_weights()                     # on_fit_start, transformer_language_model.py:74-75
        if world > 1:
            model.enable_data_parallel()
        datamodule.prepare_data()
        datamodule.setup('fit')
        model.setup('fit')
        model.on_train_start()
        [opt], [sch] = model.configure_optimizers(datamodule.tokens_per_step(), self.accumulate_grad_batches)
        sched = sch['scheduler']
        self.model, self.optimizer, self.lr_scheduler = model, opt, sched
        model.train()
        t0 = time.time()
        accum = self.accumulate_grad_batches
        done = False
        try:
            while not done and (self.max_epochs is None or self.current_epoch < self.max_epochs):
                loader = datamodule.train_dataloader()
                every = self._val_every(loader)
                it = iter(loader)
                batch = next(it, None)
                if batch is None:
                    break
                i, micro = 0, 0
                while batch is not None:
                    nxt = next(it, None)                 # one batch of lookahead: the epoch's last micro-step
                    micro += 1
                    step_now = micro == accum or nxt is None
                    model.require_backward_grad_sync = step_now
                    out = model.training_step(batch, i)
                    (out['loss'] / accum).backward()
                    model.on_after_backward()
                    if step_now:
                        opt.step()
                        sched.step()
                        opt.zero_grad()
                        micro = 0
                        self.global_step += 1
                        model.logged['loss'] = out['loss'].detach()
                        if world > 1 and hasattr(model, 'reduce_logged'):
                            model.reduce_logged()          # rank means of the logged scalars
                        if rank == 0 and self.global_step % self.log_every_n_steps == 0:
                            logs = (model.logged_values() if hasattr(model, 'logged_values')
                                    else {k: _scalar(v) for k, v in model.logged.items()})
                            logs['step'] = self.global_step
                            logs['elapsed_s'] = round(time.time() - t0, 2)
                            self.history.append(logs)
                            print(logs, flush=True)
                    i += 1
                    if every is not None and i % every == 0:
                        self.validate(model)
                        model.train()
                    if step_now and 0 < self.max_steps <= self.global_step:
                        done = True
                        break
                    batch = nxt
                if not done and every is None:
                    self.validate(model)
                    model.train()
                self.current_epoch += 1
        except KeyboardInterrupt:        # cosine_decay's end-of-schedule signal (language_model.py:139)
            pass
        finally:
            model.require_backward_grad_sync = True
        return self.history
