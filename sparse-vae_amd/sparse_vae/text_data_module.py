"""TextDataModule (text_data_module.py:19-273 in the reference) — batch wire format and a synthetic mode.

Wire format kept from the reference (collate, :194-210): {'token_ids': PaddedTensor int16 [B, L] (pad 0,
[CLS]=1 first, [SEP]=2 last, L padded to a multiple of 512), 'num_tokens': int64 [B], 'num_bytes': int64 [B]}.

The reference's only data source is HuggingFace `load_dataset` (network). Here `dataset_name='synthetic'`
generates token batches of that exact format from a fixed seed (ids uniform in [3, vocab));
a pre-tokenized dataset saved with `datasets` can be read with `dataset_path` (offline).
"""
from typing import Dict, List, Optional

import numpy as np
import torch

from .core.padded_tensor import PaddedTensor


class TextDataModule:
    def __init__(self, tokens_per_batch: Optional[int] = 50_000, chunk_documents: bool = False,
                 dataset_name: str = 'wikipedia', dataset_config: Optional[str] = '20200501.en',
                 dataset_path: Optional[str] = None, min_tokens_per_sample: int = 512,
                 max_tokens_per_sample: int = 25_000, split: Optional[str] = None, vocab_size: int = 2 ** 15,
                 seq_len: int = 512, batch_size: Optional[int] = None, padded: bool = False, seed: int = 7295,
                 num_batches: int = 1_000_000):
        from .core.language_model import AttributeDict
        self.hparams = AttributeDict(dict(
            tokens_per_batch=tokens_per_batch, chunk_documents=chunk_documents, dataset_name=dataset_name,
            dataset_config=dataset_config, dataset_path=dataset_path, min_tokens_per_sample=min_tokens_per_sample,
            max_tokens_per_sample=max_tokens_per_sample, split=split, vocab_size=vocab_size, seq_len=seq_len,
            batch_size=batch_size, padded=padded, seed=seed, num_batches=num_batches))
        self.pad_to_multiple_of = 512          # text_data_module.py:50
        self.extra_start_tokens = 0
        self.start_token = 1
        self.bytes_per_token = torch.ones(vocab_size)
        self.tokenizer = None
        self.dataset = None

    @property
    def synthetic(self):
        return self.hparams.dataset_name == 'synthetic'

    def prepare_data(self, *args, **kwargs):
        if self.synthetic:
            return
        if self.hparams.dataset_path:
            from datasets import DatasetDict
            self.dataset = DatasetDict.load_from_disk(self.hparams.dataset_path)
            return
        raise RuntimeError('the HuggingFace download path (text_data_module.py:88-96) needs the network; use '
                           "dataset_name='synthetic' or dataset_path=<pre-tokenized dataset saved to disk>")

    def setup(self, stage: Optional[str] = None):
        pass

    # ------------------------------------------------------------------ synthetic batches
    def batch_shape(self):
        L = self.hparams.seq_len
        B = self.hparams.batch_size or max(1, self.hparams.tokens_per_batch // L)
        return B, L

    def synthetic_batch(self, index: int, device=None) -> Dict[str, torch.Tensor]:
        B, L = self.batch_shape()
        rng = np.random.default_rng(self.hparams.seed + 1_000_003 * index)
        ids = rng.integers(3, self.hparams.vocab_size, size=(B, L), dtype=np.int64)
        ids[:, 0] = 1
        if self.hparams.padded:
            lens = rng.integers(L // 2, L + 1, size=B)
        else:
            lens = np.full(B, L)
        for b, n in enumerate(lens):
            ids[b, n - 1] = 2
            ids[b, n:] = 0
        seqs = [torch.from_numpy(ids[b, :n].astype(np.int16)) for b, n in enumerate(lens)]
        lens_t = torch.as_tensor(lens, dtype=torch.int64)
        batch = {'num_bytes': lens_t.clone(), 'num_tokens': lens_t, 'token_ids': PaddedTensor.from_raw(self.pad_pack(seqs))}
        if device is not None:
            raw = batch['token_ids'].as_raw().to(device)
            batch = {'token_ids': PaddedTensor.from_raw(raw), 'num_tokens': lens_t.to(device),
                     'num_bytes': lens_t.to(device)}
        return batch

    def train_dataloader(self, split: str = 'train'):
        if not self.synthetic:
            raise RuntimeError('real-data loading is the next step (SURVEY §8(f)-3); use dataset_name=synthetic')
        return (self.synthetic_batch(i) for i in range(self.hparams.num_batches))

    def val_dataloader(self):
        return (self.synthetic_batch(10 ** 9 + i) for i in range(8))

    # ------------------------------------------------------------------ reference collate semantics
    def collate(self, inputs: List[Dict]) -> Dict[str, torch.Tensor]:
        """text_data_module.py:194-210 (ids as int16 when the vocab fits)."""
        upcast = self.hparams.vocab_size > 2 ** 15
        return {
            'num_bytes': torch.tensor([x['num_bytes'] for x in inputs]),
            'num_tokens': torch.tensor([x['num_tokens'] for x in inputs]),
            'token_ids': PaddedTensor.from_raw(self.pad_pack([
                torch.from_numpy(np.asarray(x['text']).astype(np.uint16).view(np.int16) if not upcast
                                 else np.asarray(x['text']).astype(np.int32)) for x in inputs])),
        }

    def pad_pack(self, batch: List[torch.Tensor], pad_value: int = 0) -> torch.Tensor:
        """text_data_module.py:212-228: pad to the longest sequence, rounded up to a multiple of 512."""
        extras = self.extra_start_tokens
        buffer_len = max(len(x) for x in batch) + extras
        factor = self.pad_to_multiple_of
        if factor > 1 and buffer_len % factor:
            buffer_len += factor - buffer_len % factor
        buffer = torch.full([len(batch), buffer_len], pad_value, dtype=batch[0].dtype)
        if extras:
            buffer[:, :extras] = self.start_token
        for i, seq in enumerate(batch):
            buffer[i, extras:len(seq) + extras] = seq
        return buffer
