"""A minimal Trainer for the reference's fit loop (pytorch_lightning is not installed here).

Per step: training_step -> loss.backward() (engine backward; with data parallelism the bucketed RCCL
all-reduces run during it) -> on_after_backward (grad norm + KL anneal) -> RAdam.step (fused clip + update)
-> LambdaLR.step. One process per GPU: launch with torch.distributed.run; RANK/LOCAL_RANK/WORLD_SIZE come
from the environment and the backend is 'nccl' (RCCL on ROCm).
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


class Trainer:
    def __init__(self, max_steps: int = -1, accumulate_grad_batches: int = 1, log_every_n_steps: int = 50,
                 val_check_interval=None, gpus=None, precision='bf16', **unused):
        self.max_steps = max_steps
        self.accumulate_grad_batches = accumulate_grad_batches
        self.log_every_n_steps = log_every_n_steps
        self.global_step = 0
        self.datamodule = None
        self.history = []

    def fit(self, model, datamodule=None):
        world, rank, local = init_distributed()
        self.datamodule = datamodule
        model._trainer = self
        if torch.cuda.is_available():
            model.cuda()
        model.initialize_weights()                     # on_fit_start, transformer_language_model.py:74-75
        if world > 1:
            model.enable_data_parallel()
        model.on_train_start()
        datamodule.prepare_data()
        datamodule.setup('fit')
        [opt], [sch] = model.configure_optimizers(datamodule.tokens_per_step(), self.accumulate_grad_batches)
        sched = sch['scheduler']
        model.train()
        t0 = time.time()
        micro = 0
        try:
            for i, batch in enumerate(datamodule.train_dataloader()):
                if world > 1 and i % world != rank:
                    continue
                out = model.training_step(batch, i)
                loss = out['loss'] / self.accumulate_grad_batches
                loss.backward()
                model.on_after_backward()
                micro += 1
                if micro % self.accumulate_grad_batches == 0:
                    opt.step()
                    sched.step()
                    opt.zero_grad()
                    self.global_step += 1
                    if rank == 0 and self.global_step % self.log_every_n_steps == 0:
                        logs = {k: (v.item() if torch.is_tensor(v) else v) for k, v in model.logged.items()}
                        logs['step'] = self.global_step
                        logs['elapsed_s'] = round(time.time() - t0, 2)
                        self.history.append(logs)
                        print(logs, flush=True)
                    if 0 < self.max_steps <= self.global_step:
                        break
        except KeyboardInterrupt:        # cosine_decay's end-of-schedule signal (language_model.py:139)
            pass
        return self.history
