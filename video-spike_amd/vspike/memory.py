"""Arena carving: one caching-allocator request per phase, typed views at 256-B boundaries."""
from __future__ import annotations

from typing import Dict, Tuple

import torch

_ALIGN = 256


class Arena:
    """Plan named tensors, allocate them in one torch.empty, hand out views."""

    def __init__(self):
        self._plan: Dict[str, Tuple[int, Tuple[int, ...], torch.dtype]] = {}
        self._bytes = 0
        self._buf = None

    def add(self, name: str, shape, dtype: torch.dtype) -> None:
        n = 1
        for s in shape:
            n *= int(s)
        nbytes = n * dtype.itemsize
        self._plan[name] = (self._bytes, tuple(int(s) for s in shape), dtype)
        self._bytes += (nbytes + _ALIGN - 1) // _ALIGN * _ALIGN

    @property
    def nbytes(self) -> int:
        return self._bytes

    def allocate(self, device) -> Dict[str, torch.Tensor]:
        self._buf = torch.empty(max(self._bytes, _ALIGN), dtype=torch.uint8, device=device)
        out = {}
        for name, (off, shape, dtype) in self._plan.items():
            n = 1
            for s in shape:
                n *= s
            out[name] = self._buf[off:off + n * dtype.itemsize].view(dtype).view(shape)
        return out
