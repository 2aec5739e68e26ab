"""A small TensorDict: a dict of tensors sharing leading batch dims.

The reference builds its buffers on the ``tensordict`` package (not in the MI355X image).
This class implements the subset the framework needs: batch-dim indexing (int / slice /
index tensors, including assignment), view/reshape/permute/unsqueeze over batch dims,
``to(device)``, ``clone``, and ``torch.cat`` / ``torch.stack`` via ``__torch_function__``.
"""
from __future__ import annotations

from typing import Any, Dict, Iterable, Iterator, Optional, Sequence, Tuple, Union

import numpy as np
import torch
from torch import Tensor


def _as_size(bs) -> torch.Size:
    if isinstance(bs, int):
        return torch.Size([bs])
    return torch.Size(list(bs))


class TensorDict:
    def __init__(self, source: Optional[Dict[str, Any]] = None, batch_size: Sequence[int] = (), device=None):
        self._batch_size = _as_size(batch_size)
        self._device = torch.device(device) if device is not None else None
        self._data: Dict[str, Tensor] = {}
        for k, v in (source or {}).items():
            self.set(k, v)

    # ------------------------------------------------------------------ basics
    @property
    def batch_size(self) -> torch.Size:
        return self._batch_size

    @property
    def shape(self) -> torch.Size:
        return self._batch_size

    @property
    def device(self):
        return self._device

    def keys(self):
        return self._data.keys()

    def values(self):
        return self._data.values()

    def items(self):
        return self._data.items()

    def __iter__(self) -> Iterator[str]:
        return iter(self._data)

    def __contains__(self, k) -> bool:
        return k in self._data

    def __len__(self) -> int:
        return self._batch_size[0] if len(self._batch_size) else 0

    def get(self, key: str, default=None) -> Tensor:
        return self._data.get(key, default)

    def set(self, key: str, value: Any, inplace: bool = False) -> "TensorDict":
        if isinstance(value, TensorDict):
            raise TypeError("nested TensorDicts are not supported")
        if not isinstance(value, Tensor):
            value = torch.as_tensor(np.asarray(value))
        if self._device is not None and value.device != self._device:
            value = value.to(self._device)
        nb = len(self._batch_size)
        if tuple(value.shape[:nb]) != tuple(self._batch_size):
            try:
                value = value.expand(*self._batch_size, *value.shape[nb:]) if value.dim() >= nb else value
            except RuntimeError:
                pass
            if tuple(value.shape[:nb]) != tuple(self._batch_size):
                raise RuntimeError(f"batch dimension mismatch for key '{key}': got {tuple(value.shape)}, expected leading {tuple(self._batch_size)}")
        if inplace and key in self._data:
            self._data[key].copy_(value)
        else:
            self._data[key] = value
        return self

    def update(self, other: Union["TensorDict", Dict[str, Any]]) -> "TensorDict":
        for k, v in other.items():
            self.set(k, v)
        return self

    def pop(self, key: str, *default):
        return self._data.pop(key, *default)

    def to_dict(self) -> Dict[str, Tensor]:
        return dict(self._data)

    def __repr__(self) -> str:
        fields = ", ".join(f"{k}: {tuple(v.shape)} {v.dtype}" for k, v in self._data.items())
        return f"TensorDict(batch_size={tuple(self._batch_size)}, device={self._device}, {{{fields}}})"

    # ------------------------------------------------------------------ indexing
    def _index_batch(self, idx) -> Tuple[Any, torch.Size]:
        probe = torch.empty(self._batch_size, device="meta")
        return idx, probe[idx].shape

    def __getitem__(self, idx):
        if isinstance(idx, str):
            return self._data[idx]
        idx_n = self._normalize_index(idx)
        nb = len(self._batch_size)
        data = {k: v[idx_n] for k, v in self._data.items()}
        if data:
            k0 = next(iter(data))
            feat = self._data[k0].dim() - nb
            shp = data[k0].shape
            new_bs = shp[: len(shp) - feat]
        else:
            _, new_bs = self._index_batch(self._cpu_index(idx_n))
        out = TensorDict(batch_size=new_bs, device=self._device)
        out._data = data
        return out

    @staticmethod
    def _cpu_index(idx):
        if isinstance(idx, tuple):
            return tuple(i.cpu() if isinstance(i, Tensor) else i for i in idx)
        return idx.cpu() if isinstance(idx, Tensor) else idx

    def _normalize_index(self, idx):
        if isinstance(idx, tuple):
            dev = self._first_device()
            return tuple((i.to(dev) if isinstance(i, Tensor) and i.device != dev else i) for i in idx)
        if isinstance(idx, Tensor) and idx.device != self._first_device():
            return idx.to(self._first_device())
        return idx

    def _first_device(self):
        for v in self._data.values():
            return v.device
        return self._device or torch.device("cpu")

    def __setitem__(self, idx, value) -> None:
        if isinstance(idx, str):
            self.set(idx, value)
            return
        idx_n = self._normalize_index(idx)
        items = value.items() if isinstance(value, (TensorDict, dict)) else None
        if items is None:
            raise TypeError("can only assign a TensorDict/dict to a TensorDict slice")
        for k, v in items:
            if k not in self._data:
                raise KeyError(f"key '{k}' not in the destination TensorDict")
            dst = self._data[k]
            dst[idx_n] = v.to(dst.device, dst.dtype) if isinstance(v, Tensor) else torch.as_tensor(v, dtype=dst.dtype)

    # ------------------------------------------------------------------ shape ops
    def _apply(self, fn, new_bs) -> "TensorDict":
        out = TensorDict(batch_size=new_bs, device=self._device)
        for k, v in self._data.items():
            out._data[k] = fn(v)
        return out

    def view(self, *shape) -> "TensorDict":
        if len(shape) == 1 and isinstance(shape[0], (tuple, list, torch.Size)):
            shape = tuple(shape[0])
        nb = len(self._batch_size)
        new_bs = torch.empty(self._batch_size, device="meta").view(*shape).shape
        return self._apply(lambda v: v.reshape(*new_bs, *v.shape[nb:]), new_bs)

    reshape = view

    def permute(self, *dims) -> "TensorDict":
        if len(dims) == 1 and isinstance(dims[0], (tuple, list)):
            dims = tuple(dims[0])
        nb = len(self._batch_size)
        dims = tuple(d % nb for d in dims)
        new_bs = torch.Size([self._batch_size[d] for d in dims])
        return self._apply(lambda v: v.permute(*dims, *range(nb, v.dim())), new_bs)

    def unsqueeze(self, dim: int) -> "TensorDict":
        nb = len(self._batch_size)
        d = dim if dim >= 0 else nb + dim + 1
        bs = list(self._batch_size)
        bs.insert(d, 1)
        return self._apply(lambda v: v.unsqueeze(d), torch.Size(bs))

    def squeeze(self, dim: int) -> "TensorDict":
        nb = len(self._batch_size)
        d = dim % nb
        bs = list(self._batch_size)
        bs.pop(d)
        return self._apply(lambda v: v.squeeze(d), torch.Size(bs))

    def flatten(self, start: int = 0, end: int = -1) -> "TensorDict":
        nb = len(self._batch_size)
        s, e = start % nb, end % nb
        bs = list(self._batch_size)
        n = int(np.prod(bs[s : e + 1]))
        new_bs = torch.Size(bs[:s] + [n] + bs[e + 1 :])
        return self.view(*new_bs)

    def to(self, device, non_blocking: bool = False) -> "TensorDict":
        device = torch.device(device)
        out = TensorDict(batch_size=self._batch_size, device=device)
        for k, v in self._data.items():
            out._data[k] = v.to(device, non_blocking=non_blocking)
        return out

    def clone(self) -> "TensorDict":
        return self._apply(lambda v: v.clone(), self._batch_size)

    def float(self) -> "TensorDict":
        return self._apply(lambda v: v.float(), self._batch_size)

    def detach(self) -> "TensorDict":
        return self._apply(lambda v: v.detach(), self._batch_size)

    def apply(self, fn) -> "TensorDict":
        return self._apply(fn, self._batch_size)

    # ------------------------------------------------------------------ torch.cat / torch.stack
    @classmethod
    def __torch_function__(cls, func, types, args=(), kwargs=None):
        kwargs = kwargs or {}
        if func in (torch.cat, torch.concat, torch.concatenate):
            tds = list(args[0])
            dim = kwargs.get("dim", args[1] if len(args) > 1 else 0)
            return cat(tds, dim)
        if func is torch.stack:
            tds = list(args[0])
            dim = kwargs.get("dim", args[1] if len(args) > 1 else 0)
            return stack(tds, dim)
        return NotImplemented


def cat(tds: Sequence[TensorDict], dim: int = 0) -> TensorDict:
    nb = len(tds[0].batch_size)
    d = dim % nb
    keys = list(tds[0].keys())
    bs = list(tds[0].batch_size)
    bs[d] = sum(t.batch_size[d] for t in tds)
    out = TensorDict(batch_size=bs, device=tds[0].device)
    for k in keys:
        out._data[k] = torch.cat([t[k] for t in tds], dim=d)
    return out


def stack(tds: Sequence[TensorDict], dim: int = 0) -> TensorDict:
    nb = len(tds[0].batch_size)
    d = dim % (nb + 1)
    bs = list(tds[0].batch_size)
    bs.insert(d, len(tds))
    out = TensorDict(batch_size=bs, device=tds[0].device)
    for k in tds[0].keys():
        out._data[k] = torch.stack([t[k] for t in tds], dim=d)
    return out


def pad_sequence(seqs: Sequence[TensorDict], return_mask: bool = True) -> TensorDict:
    """Stack variable-length ``[L_i, ...]`` TensorDicts into ``[L_max, N, ...]`` (zero padding at
    the END of each sequence) plus a boolean ``mask`` ``[L_max, N]`` (True on real steps)."""
    if not seqs:
        raise ValueError("pad_sequence needs at least one sequence")
    L = max(s.shape[0] for s in seqs)
    N = len(seqs)
    dev = seqs[0]._first_device()
    out = {}
    for k in seqs[0].keys():
        ref = seqs[0][k]
        buf = torch.zeros((L, N) + tuple(ref.shape[1:]), dtype=ref.dtype, device=ref.device)
        for i, s in enumerate(seqs):
            buf[: s.shape[0], i] = s[k]
        out[k] = buf
    if return_mask:
        lengths = torch.tensor([s.shape[0] for s in seqs], device=dev)
        out["mask"] = torch.arange(L, device=dev).unsqueeze(1) < lengths.unsqueeze(0)
    return TensorDict(out, batch_size=[L, N], device=dev)
