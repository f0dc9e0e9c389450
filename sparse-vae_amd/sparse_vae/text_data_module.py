"""TextDataModule (text_data_module.py:19-273 in the reference) — batch wire format, a synthetic mode and the
real-data path run offline.

Wire format kept from the reference (collate, :194-210): {'token_ids': PaddedTensor int16 [B, L] (pad 0,
[CLS]=1 first, [SEP]=2 last, L padded to a multiple of 512), 'num_tokens': int64 [B], 'num_bytes': int64 [B]}.

Data sources:
* `dataset_name='synthetic'`: batches of that exact format from a fixed seed (ids uniform in [3, vocab),
  SURVEY §8(d)).
* `dataset_path=<DatasetDict saved with save_to_disk>`: the reference's real-data path (:98-228) without the
  network. Raw 'text' is tokenised by the byte-level BPE tokenizer in
  ./sparse-vae-pretrained/tokenizers/<dataset_name>.json (trained on the train split and saved there when
  absent; [PAD]=0 [CLS]=1 [SEP]=2), a pre-tokenised integer 'text' column is used as is; documents are filtered
  to [min_tokens_per_sample, max_tokens_per_sample], split off a test set (5 %, at most 50k) when there is none,
  binned to multiples of 512 and packed into token-budget batches by UniformSizeRandomSampler.
The HuggingFace download (:93-96) needs the network and raises.
"""
import os
from pathlib import Path
from typing import Dict, List, Optional

import numpy as np
import torch

from .core.padded_tensor import PaddedTensor
from .data_utils import UniformSizeRandomSampler, get_features_all_equal, length_bins, tokenize


class TextDataModule:
    def __init__(self, tokens_per_batch: Optional[int] = 50_000, chunk_documents: bool = False,
                 dataset_name: str = 'wikipedia', dataset_config: Optional[str] = '20200501.en',
                 dataset_path: Optional[str] = None, min_tokens_per_sample: int = 512,
                 max_tokens_per_sample: int = 25_000, split: Optional[str] = None, vocab_size: int = 2 ** 15,
                 seq_len: int = 512, batch_size: Optional[int] = None, padded: bool = False, seed: int = 7295,
                 num_batches: int = 1_000_000, num_workers: int = 10):
        from .core.language_model import AttributeDict
        self.hparams = AttributeDict(dict(
            tokens_per_batch=tokens_per_batch, chunk_documents=chunk_documents, dataset_name=dataset_name,
            dataset_config=dataset_config, dataset_path=dataset_path, min_tokens_per_sample=min_tokens_per_sample,
            max_tokens_per_sample=max_tokens_per_sample, split=split, vocab_size=vocab_size, seq_len=seq_len,
            batch_size=batch_size, padded=padded, seed=seed, num_batches=num_batches, num_workers=num_workers))
        self.pad_to_multiple_of = 512          # text_data_module.py:50
        self.extra_start_tokens = 0
        self.start_token = 1
        self.bytes_per_token = torch.ones(vocab_size)
        self._tokenizer = None
        self.dataset = None

    @property
    def synthetic(self):
        return self.hparams.dataset_name == 'synthetic'

    # ------------------------------------------------------------------ real data (offline)
    def create_dataset(self):
        """text_data_module.py:88-96 without the network: a Dataset / DatasetDict saved to disk."""
        if not self.hparams.dataset_path:
            raise RuntimeError('the HuggingFace download path (text_data_module.py:93-96) needs the network; use '
                               "dataset_name='synthetic' or dataset_path=<DatasetDict saved with save_to_disk>")
        from datasets import load_from_disk
        self.dataset = load_from_disk(self.hparams.dataset_path)

    @property
    def tokenizer(self):
        if self._tokenizer is None:
            self.setup_tokenizer()
        return self._tokenizer

    def setup_tokenizer(self):
        """text_data_module.py:231-273: load ./sparse-vae-pretrained/tokenizers/<name>.json, or train a byte-level
        BPE ([CLS] ... [SEP] post-processing) on the train split and save it there; then the bytes per token of
        the bits-per-byte metric (special tokens count as 1 byte)."""
        from tokenizers import Tokenizer
        from tokenizers.implementations import ByteLevelBPETokenizer
        from tokenizers.processors import RobertaProcessing
        tok_dir = Path.cwd() / 'sparse-vae-pretrained' / 'tokenizers'
        tok_dir.mkdir(parents=True, exist_ok=True)
        path = tok_dir / (self.hparams.dataset_name + '.json')
        if path.exists():
            self._tokenizer = Tokenizer.from_file(str(path))
            assert self._tokenizer.get_vocab_size() == self.hparams.vocab_size
        else:
            tok = ByteLevelBPETokenizer()
            tok.post_processor = RobertaProcessing(sep=('[SEP]', 2), cls=('[CLS]', 1))
            data = self.dataset['train'] if hasattr(self.dataset, 'keys') else self.dataset
            step = 1000

            def texts():
                for i in range(0, len(data), step):
                    yield data[i:i + step]['text']

            tok.train_from_iterator(texts(), vocab_size=self.hparams.vocab_size,
                                    special_tokens=['[PAD]', '[CLS]', '[SEP]'])
            tok.save(str(path))
            self._tokenizer = tok
        for token, tid in self._tokenizer.get_vocab().items():
            if tid < len(self.bytes_per_token):
                self.bytes_per_token[tid] = len(token.encode()) if tid > 2 else 1
        self.start_token = self._tokenizer.get_vocab()['[CLS]']
        if self.hparams.chunk_documents:
            self._tokenizer.enable_truncation(self.hparams.max_tokens_per_sample)

    def prepare_data(self, *args, **kwargs):
        """text_data_module.py:98-170."""
        if self.synthetic:
            return
        self.create_dataset()
        feats = get_features_all_equal(self.dataset)
        text = feats.get('text')
        assert text is not None, "Can't find text column in dataset"
        if str(getattr(getattr(text, 'feature', None), 'dtype', '')).startswith(('int', 'uint')):   # pre-tokenised
            self.dataset = self.dataset.map(lambda b: {'num_tokens': [len(r) for r in b['text']]}, batched=True,
                                            batch_size=1000)
        else:
            from datasets import Features, Sequence, Value
            ftypes = {'num_bytes': Value('int32'), 'num_tokens': Value('int32'), 'text': Sequence(Value('uint16'))}
            for extra, t in (('title', Value('string')), ('label', Value('uint8'))):
                if extra in feats:
                    ftypes[extra] = t
            self.dataset = self.dataset.map(tokenize, batched=True, batch_size=1000, features=Features(ftypes),
                                            fn_kwargs=dict(chunk=self.hparams.chunk_documents,
                                                           tokenizer=self.tokenizer))
        lo, hi = self.hparams.min_tokens_per_sample, self.hparams.max_tokens_per_sample
        self.dataset = self.dataset.filter(lambda n: lo <= n <= hi, input_columns='num_tokens')
        from datasets import DatasetDict
        if not isinstance(self.dataset, DatasetDict):
            n = len(self.dataset)
            self.dataset = self.dataset.train_test_split(test_size=min(50_000, max(1, round(n * 0.05))), shuffle=True)
        elif 'test' not in self.dataset:
            n = len(self.dataset['train'])
            self.dataset = self.dataset['train'].train_test_split(test_size=min(50_000, max(1, round(n * 0.05))),
                                                                  shuffle=True)
        bins = self.pad_to_multiple_of
        self.dataset = self.dataset.map(lambda b: {'length_bin': length_bins(b['num_tokens'], bins)}, batched=True)

    def setup(self, stage: Optional[str] = None):
        if not self.synthetic and self.dataset is not None:
            self.dataset.set_format('numpy')    # collate reinterprets the uint16 ids itself

    def tokens_per_step(self) -> int:
        """Tokens per batch for the learning-rate scaling of configure_optimizers (language_model.py:68-78):
        the synthetic batch's B x L, else the token budget."""
        if self.synthetic:
            B, L = self.batch_shape()
            return B * L
        return int(self.hparams.tokens_per_batch)

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

    # ------------------------------------------------------------------ loaders
    @staticmethod
    def _rank_world(rank=None, world=None):
        if rank is None or world is None:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                return dist.get_rank(), dist.get_world_size()
            return 0, 1
        return rank, world

    def train_dataloader(self, split: str = 'train', rank: Optional[int] = None, world: Optional[int] = None):
        """text_data_module.py:176-184: token-budget batches of similar-length documents, collated in worker
        processes into pinned memory. Under data parallelism (an initialised process group, or rank/world given)
        rank r gets batches r, r + world, ... of the first len - len % world: disjoint shards, equal counts."""
        rank, world = self._rank_world(rank, world)
        if self.synthetic:
            n = self.hparams.num_batches if split == 'train' else 8
            base = 0 if split == 'train' else 10 ** 9
            return _SyntheticLoader(self, base, n - n % world if world > 1 else n, rank, world)
        from torch.utils.data import DataLoader
        if self.dataset is None:
            self.prepare_data()
            self.setup()
        data = self.dataset[split]
        docs = list(enumerate(np.asarray(data['length_bin']).tolist()))
        sampler = UniformSizeRandomSampler(documents=docs, max_size=self.hparams.tokens_per_batch)
        if world > 1:
            sampler = RankBatchSampler(sampler, rank, world)
        workers = min(self.hparams.num_workers, os.cpu_count() or 1)
        return DataLoader(data, batch_sampler=sampler, collate_fn=self.collate, num_workers=workers,
                          pin_memory=torch.cuda.is_available())

    def val_dataloader(self, rank: Optional[int] = None, world: Optional[int] = None):
        return self.train_dataloader(split='test' if not self.synthetic else 'val', rank=rank, world=world)

    def test_dataloader(self, *args, **kwargs):
        return self.val_dataloader()

    # ------------------------------------------------------------------ reference collate semantics
    def collate(self, inputs: List[Dict]) -> Dict[str, torch.Tensor]:
        """text_data_module.py:194-210 (ids reinterpreted as int16 when the vocab fits, else int32)."""
        upcast = self.hparams.vocab_size > 2 ** 15
        batch = {
            'num_bytes': torch.tensor([int(x['num_bytes'] if 'num_bytes' in x else x['num_tokens']) for x in inputs]),
            'num_tokens': torch.tensor([int(x['num_tokens']) for x in inputs]),
            'token_ids': PaddedTensor.from_raw(self.pad_pack([
                torch.from_numpy(np.asarray(x['text']).astype(np.uint16).view(np.int16) if not upcast
                                 else np.asarray(x['text']).astype(np.int32)) for x in inputs])),
        }
        if 'label' in inputs[0]:
            batch['label'] = torch.tensor([int(x['label']) for x in inputs])
        return batch

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


class _SyntheticLoader:
    """Synthetic batches base + k for k = rank, rank + world, ... < n (a sized iterable, one pass)."""

    def __init__(self, dm, base, n, rank, world):
        self.dm, self.base, self.n, self.rank, self.world = dm, base, n, rank, world

    def __len__(self):
        return len(range(self.rank, self.n, self.world))

    def __iter__(self):
        return (self.dm.synthetic_batch(self.base + k) for k in range(self.rank, self.n, self.world))


class RankBatchSampler:
    """Data-parallel shard of a batch sampler: rank r takes batches r, r + world, ... of each epoch's first
    len - len % world batches, so every rank runs the same number of steps (and collectives). Every rank draws
    the same batch order (seed_everything on all ranks), as Lightning's replaced samplers assume."""

    def __init__(self, sampler, rank, world):
        self.sampler, self.rank, self.world = sampler, rank, world

    def __len__(self):
        return len(self.sampler) // self.world

    def __iter__(self):
        n = len(self.sampler) // self.world * self.world
        for i, b in enumerate(self.sampler):
            if i >= n:
                continue                      # drain the epoch (the sampler repacks when exhausted)
            if i % self.world == self.rank:
                yield b
