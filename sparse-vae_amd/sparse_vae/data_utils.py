"""Host-side data plumbing of the real-data TextDataModule path (reference: sparse_vae/data_utils.py).

Tokenisation with per-document statistics, token-budget batching (documents sorted by padded length so a
batch wastes little padding), and the dataset-shape helpers. Pure host code: the batches it produces are the
same wire format the synthetic mode makes (collate -> PaddedTensor int16 [B, L]).
"""
import random
from dataclasses import dataclass, field
from itertools import chain
from typing import Dict, List, Tuple, Union

import numpy as np

try:   # torch's Sampler base only adds __len__/__iter__ typing; keep the module importable without it
    from torch.utils.data.sampler import Sampler
except Exception:  # pragma: no cover
    Sampler = object


def tokenize(batch, tokenizer, chunk: bool) -> Dict[str, list]:
    """data_utils.py:12-25: encode a batch of raw texts; with `chunk`, overflowing pieces (the tokenizer's
    truncation windows) become documents of their own. Records token ids, UTF-8 byte counts and token counts."""
    texts = batch['text']
    encs = tokenizer.encode_batch(texts)
    if chunk:
        encs = list(chain.from_iterable([e] + list(e.overflowing) for e in encs))
    ids = [e.ids for e in encs]
    return {'text': ids, 'num_bytes': [len(t.encode('utf8')) for t in texts], 'num_tokens': [len(x) for x in ids]}


def length_bins(num_tokens, bin_size: int) -> np.ndarray:
    """text_data_module.py:164-170: round each count UP to the next multiple of bin_size. As in the reference,
    an exact multiple still moves up one whole bin (n + (bin - n % bin))."""
    n = np.asarray(num_tokens, dtype=np.int64)
    return n + (bin_size - n % bin_size)


@dataclass
class PrebatchedRandomSampler:
    """data_utils.py:28-49: iterate precomputed (start, length) contiguous batches in random order; one pass
    per epoch, reshuffled when exhausted."""
    batches: List[Tuple[int, int]]
    _left: list = field(default_factory=list, init=False, repr=False)

    def __post_init__(self):
        self._reshuffle()

    def _reshuffle(self):
        self._left = list(self.batches)
        random.shuffle(self._left)

    def __iter__(self):
        return self

    def __len__(self):
        return len(self.batches)

    def __next__(self):
        if not self._left:
            self._reshuffle()
            raise StopIteration
        start, length = self._left.pop()
        assert length > 0, 'zero-length batch'
        return list(range(start, start + length))


@dataclass
class UniformSizeRandomSampler(Sampler):
    """data_utils.py:52-97: batches of document indices whose padded size (longest length bin x count) stays
    within `max_size` tokens. Documents are shuffled, then stably sorted by length bin (so each bin is shuffled
    internally), packed greedily in that order, and the batches visited in random order."""
    documents: List[Tuple[int, int]]    # (document index, length bin)
    max_size: int

    def __post_init__(self):
        assert all(n <= self.max_size for _, n in self.documents), 'a document exceeds tokens_per_batch'
        self._pack()

    def _pack(self):
        random.shuffle(self.documents)
        self.documents.sort(key=lambda d: d[1])
        batches, cur, longest = [], [], 0
        for idx, n in self.documents:
            if cur and max(longest, n) * (len(cur) + 1) > self.max_size:
                batches.append(cur)
                cur, longest = [], 0
            cur.append(idx)
            longest = max(longest, n)
        batches.append(cur)
        random.shuffle(batches)
        self.batches = batches

    def __iter__(self):
        return self

    def __len__(self):
        return len(self.batches)

    def __next__(self):
        if not self.batches:
            self._pack()
            raise StopIteration
        batch = self.batches.pop()
        assert batch, 'zero-length batch'
        return batch


def get_columns_all_equal(dataset) -> List[str]:
    """data_utils.py:100-109: column names, identical across the splits of a DatasetDict."""
    if hasattr(dataset, 'column_names') and isinstance(dataset.column_names, dict):
        cols = list(dataset.column_names.values())
        assert all(c == cols[0] for c in cols), 'All splits must have the same columns'
        return cols[0]
    return dataset.column_names


def get_features_all_equal(dataset) -> dict:
    """data_utils.py:112-121: features, identical across the splits of a DatasetDict."""
    if hasattr(dataset, 'values') and not hasattr(dataset, 'features'):
        feats = [split.features for split in dataset.values()]
        assert all(f == feats[0] for f in feats), 'All splits must have the same features'
        return feats[0]
    return dataset.features


def total_dataset_len(dataset) -> int:
    """data_utils.py:123-124."""
    if hasattr(dataset, 'values') and not hasattr(dataset, 'features'):
        return sum(len(s) for s in dataset.values())
    return len(dataset)


def compute_uniform_sized_batches(lengths: List[int], max_size: int) -> Dict[str, list]:
    """data_utils.py:126-140: contiguous runs of documents whose summed length stays within max_size:
    {'start': run starts, 'length': run lengths}."""
    starts, total = [0], 0
    for i, n in enumerate(lengths):
        assert n <= max_size, f'a document has {n} tokens > max tokens per batch {max_size}'
        total += n
        if total > max_size:
            starts.append(i)
            total = n
    return {'start': starts, 'length': np.diff(starts, append=len(lengths))}
