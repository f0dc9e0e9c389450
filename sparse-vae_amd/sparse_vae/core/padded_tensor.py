"""PaddedTensor (padded_tensor.py:12-82 in the reference): a token-id tensor that carries its padding mask.

As in the reference, every torch op on a PaddedTensor returns PaddedTensors that carry the same mask (so the
mask survives `.to(device)`, `.pin_memory()`, `.long()`, slicing of the batch dict by the DataLoader, ...). The
mask is moved to the data's device lazily, and the getter returns None when it does not fit the data's
trailing dimension (the reference's key-length rule, :67-69). Only the batch boundary reads it here: the
training step hands it to the kernels as an explicit uint8 key mask.
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
        kwargs = kwargs or {}
        src = next((a for a in list(args) + list(kwargs.values()) if isinstance(a, PaddedTensor)), None)
        with torch._C.DisableTorchFunctionSubclass():
            out = func(*args, **kwargs)
        mask = getattr(src, '_padding', None) if src is not None else None

        def wrap(x):
            if isinstance(x, Tensor) and not isinstance(x, PaddedTensor):
                y = x.as_subclass(PaddedTensor)
                y._padding = mask
                return y
            return x

        if func in (Tensor.__repr__, Tensor.__str__, Tensor.__format__) or src is None:
            return out
        if isinstance(out, Tensor):
            return wrap(out)
        if isinstance(out, tuple) and not hasattr(out, '_fields'):
            return tuple(wrap(x) for x in out)
        return out

    @property
    def padding(self) -> Optional[Tensor]:
        pad = getattr(self, '_padding', None)
        if pad is None:
            return None
        with torch._C.DisableTorchFunctionSubclass():
            if pad.device != self.device:
                pad = self._padding = pad.to(self.device)
            if pad.shape[0] != self.shape[0] and pad.shape[0] == 1:
                return pad.expand(self.shape[0], *pad.shape[1:])
            return pad if pad.ndim <= self.ndim and pad.shape[-1] == self.shape[pad.ndim - 1] else None

    @padding.setter
    def padding(self, value: Optional[Tensor]):
        if value is not None:
            assert value.ndim <= self.ndim, 'Padding cannot have more dimensions than the tensor itself'
            for dim, (p, s) in enumerate(zip(value.shape, self.shape)):
                assert p == s, f'Padding size {p} must match data size {s} at dim {dim}'
            with torch._C.DisableTorchFunctionSubclass():
                value = value.to(self.device)
        self._padding = value
