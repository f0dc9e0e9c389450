"""GenerationState (generation.py in the reference): the sampling state of TransformerVAE.sample, on the device.

Same fields, defaults and methods as the reference dataclass (top_k 0, top_p 0.9, temperature 1.0,
repetition_penalty 1.2; prev_tokens / process_logits / should_stop / final_output). `process_logits` runs the
repetition penalty and the greedy / top-k / nucleus + multinomial choice as two libsvae kernels
(svae_dec_penalty, svae_dec_sample) that write output_ids and the live mask in place; the current index is
mirrored in a device int32 (`cur`) so a captured decode step reads it at run time.

Randomness: the multinomial draw uses a counter-based RNG keyed by (seed, current_index, row), with the seed
taken from torch's default generator at construction (so torch.manual_seed makes sampling reproducible); it
is not torch's Philox stream, so sampled (non-greedy) sequences differ from the reference's draw for draw.
"""
from dataclasses import InitVar, dataclass

import torch

from .. import kernels as K


@dataclass
class GenerationState:
    max_length: InitVar[int]
    batch_size: InitVar[int]
    start_token: int
    end_token: int
    device: InitVar[torch.device]
    dtype: InitVar[torch.dtype] = torch.long

    top_k: int = 0
    top_p: float = 0.9
    temperature: float = 1.0
    repetition_penalty: float = 1.2

    def __post_init__(self, max_length: int, batch_size: int, device, dtype):
        if dtype != torch.long:
            raise ValueError('output_ids are int64 on the device (the kernels write int64 ids)')
        device = torch.device(device)
        if device.type != 'cuda':
            raise RuntimeError('GenerationState runs on the MI355X kernels: pass a GPU device (no CPU fallback)')
        self.output_ids = torch.zeros(batch_size, max_length, device=device, dtype=torch.long)
        self.output_ids[:, 0] = self.start_token
        self.live_sample_mask = torch.ones(batch_size, device=device, dtype=torch.bool)
        self.cur = torch.ones(1, device=device, dtype=torch.int32)          # current_index on the device
        self.live_count = torch.full((1,), batch_size, device=device, dtype=torch.int32)
        self.seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self._index = 1

    @property
    def current_index(self) -> int:
        return self._index

    @current_index.setter
    def current_index(self, value: int):
        self._index = int(value)
        self.cur.fill_(self._index)

    def prev_tokens(self):
        return self.output_ids[self.live_sample_mask, self.current_index - 1, None]

    def process_logits(self, logits):
        """logits [n_live, V] f32 for the live rows (in row order): penalise, choose, write output_ids at the
        current index, advance it, update the live mask. Returns the continuing mask of those rows.
        The logits are modified in place (the reference penalises and rescales them in place too)."""
        if logits.dtype != torch.float32:
            logits = logits.float()
        logits = logits.contiguous()
        rows = self.live_sample_mask.nonzero().flatten().to(torch.int32)
        n = rows.numel()
        assert logits.shape[0] == n, 'process_logits expects one logits row per live sample'
        T = self.output_ids.shape[1]
        if self.repetition_penalty > 1.0:
            K.dec_penalty(logits, n, rows, self.output_ids, T, self.cur, None, float(self.repetition_penalty))
        K.dec_sample(logits, logits.shape[1], n, rows, self.output_ids, T, self.cur, self.live_sample_mask,
                     int(self.end_token), float(self.temperature), int(self.top_k), float(self.top_p), self.seed,
                     self.live_count)
        self.current_index += 1
        return self.live_sample_mask[rows.long()]

    def step_done(self):
        """Host bookkeeping after a decode step that advanced `cur` on the device itself."""
        self._index += 1

    def should_stop(self) -> bool:
        return self.current_index >= self.output_ids.shape[-1] - 1 or not bool(self.live_sample_mask.any())

    def final_output(self):
        return self.output_ids[:, 1:]
