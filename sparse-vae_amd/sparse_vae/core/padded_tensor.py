"""PaddedTensor (padded_tensor.py:12-82 in the reference): a token-id tensor that carries its padding mask.

The reference propagates the mask through every torch op via __torch_function__ so that it reaches
Attention.forward (attention.py:75). Here the mask is read ONCE, at the batch boundary, by the training
step (the kernels take it as an explicit uint8 key mask), so the subclass only has to carry it.
"""
from typing import Optional

import torch
from torch import Tensor


class PaddedTensor(Tensor):
    @classmethod
    def from_raw(cls, data: Tensor, padding: Optional[Tensor] = None) -> 'PaddedTensor':
        t = data.as_subclass(cls)
        t.padding = padding if padding is not None else data.eq(0)
        return t

    @classmethod
    def unpadded(cls, data: Tensor) -> 'PaddedTensor':
        t = data.as_subclass(cls)
        t._padding = None
        return t

    def as_raw(self) -> Tensor:
        return self.as_subclass(Tensor)

    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        # plain tensors out: the mask does not follow arithmetic (the step reads it at the boundary)
        with torch._C.DisableTorchFunctionSubclass():
            return func(*args, **(kwargs or {}))

    @property
    def padding(self) -> Optional[Tensor]:
        return getattr(self, '_padding', None)

    @padding.setter
    def padding(self, value: Optional[Tensor]):
        if value is not None:
            assert value.ndim <= self.ndim, 'Padding cannot have more dimensions than the tensor itself'
            for dim, (p, s) in enumerate(zip(value.shape, self.shape)):
                assert p == s, f'Padding size {p} must match data size {s} at dim {dim}'
        self._padding = value
