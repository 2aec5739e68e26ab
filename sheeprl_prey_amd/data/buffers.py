"""Replay buffers (reference: ``sheeprl/data/buffers.py:16-690``).

Same sampling semantics as the reference (avoid the write head, sequences never straddle it,
per-env async buffers, whole-episode buffer with FIFO eviction and ``prioritize_ends``), with
MI355X-minded storage choices:

* ``device="cuda"`` keeps the whole store resident in HBM (288 GB/GPU holds e.g. 1M 64x64x3
  uint8 frames in 12 GB) so a training sample is an on-device gather - no host->device copy
  per gradient step;
* valid start indices are drawn arithmetically on the buffer's device instead of
  materialising Python ``list(range(...))`` of up to ``buffer_size`` elements per sample;
* ``memmap=True`` stores host buffers in ``numpy.memmap`` files under ``memmap_dir``.

Buffers expose ``state_dict()`` / ``load_state_dict()`` (plain tensors) for checkpoints.
"""
from __future__ import annotations

import os
import shutil
import uuid
import warnings
from pathlib import Path
from typing import Dict, List, Optional, Sequence, Union

import numpy as np
import torch
from torch import Size, Tensor

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.data.tensordict import TensorDict, cat

_NP_DTYPES = {
    torch.float32: np.float32, torch.float64: np.float64, torch.float16: np.float16, torch.uint8: np.uint8,
    torch.int8: np.int8, torch.int16: np.int16, torch.int32: np.int32, torch.int64: np.int64, torch.bool: np.bool_,
}


def _alloc(shape, dtype, device, memmap: bool, path: Optional[Path]) -> Tensor:
    if memmap and torch.device(device).type == "cpu":
        if path is None:
            import tempfile

            fd, fname = tempfile.mkstemp(suffix=".memmap")
            os.close(fd)
            path = Path(fname)
        arr = np.memmap(str(path), dtype=_NP_DTYPES[dtype], mode="w+", shape=tuple(shape))
        return torch.from_numpy(arr)
    return torch.zeros(tuple(shape), dtype=dtype, device=device)


def _sample_two_ranges(n1: int, start2: int, n2: int, size: int, device) -> Tensor:
    """Uniform draws from [0, n1) U [start2, start2 + n2)."""
    k = torch.randint(0, n1 + n2, (size,), device=device)
    return torch.where(k < n1, k, start2 + (k - n1))


class ReplayBuffer:
    def __init__(
        self,
        buffer_size: int,
        n_envs: int = 1,
        device: Union[torch.device, str] = "cpu",
        memmap: bool = False,
        memmap_dir: Optional[Union[str, os.PathLike]] = None,
        obs_keys: Sequence[str] = ("observations",),
    ):
        if buffer_size <= 0:
            raise ValueError(f"The buffer size must be greater than zero, got: {buffer_size}")
        if n_envs <= 0:
            raise ValueError(f"The number of environments must be greater than zero, got: {n_envs}")
        self._buffer_size = buffer_size
        self._n_envs = n_envs
        self._device = torch.device(device) if isinstance(device, str) else device
        self._memmap = memmap
        self._memmap_dir = memmap_dir
        if self._memmap:
            if memmap_dir is None:
                warnings.warn(
                    "The buffer will be memory-mapped into the `/tmp` folder, this means that there is the"
                    " possibility to lose the saved files. Set the `memmap_dir` to a known directory.",
                    UserWarning,
                )
            else:
                self._memmap_dir = Path(self._memmap_dir)
                self._memmap_dir.mkdir(parents=True, exist_ok=True)
            self._buf: Optional[TensorDict] = None
        else:
            self._buf = TensorDict({}, batch_size=[buffer_size, n_envs], device=self._device)
        self._pos = 0
        self._full = False
        self.obs_keys = obs_keys

    # ------------------------------------------------------------------ properties
    @property
    def buffer(self) -> Optional[TensorDict]:
        return self._buf

    @property
    def buffer_size(self) -> int:
        return self._buffer_size

    @property
    def full(self) -> bool:
        return self._full

    @property
    def n_envs(self) -> int:
        return self._n_envs

    @property
    def shape(self) -> Optional[Size]:
        return None if self._buf is None else self._buf.shape

    @property
    def device(self) -> torch.device:
        return self._device

    @property
    def is_memmap(self) -> bool:
        return self._memmap

    @property
    def empty(self) -> bool:
        return (self._buf is None or len(self._buf.keys()) == 0) or (not self._full and self._pos == 0)

    def __len__(self) -> int:
        return self.buffer_size

    def keys(self):
        return [] if self._buf is None else list(self._buf.keys())

    # ------------------------------------------------------------------ add
    def _ensure_storage(self, data: TensorDict) -> None:
        if self._buf is None:
            self._buf = TensorDict({}, batch_size=[self._buffer_size, self._n_envs], device=self._device)
        for k, v in data.items():
            if k not in self._buf.keys():
                path = None if self._memmap_dir is None else Path(self._memmap_dir) / f"{k.replace('/', '_')}.memmap"
                self._buf._data[k] = _alloc((self._buffer_size, self._n_envs, *v.shape[2:]), v.dtype, self._device,
                                            self._memmap, path)

    def add(self, data: Union["ReplayBuffer", TensorDict]) -> None:
        if isinstance(data, ReplayBuffer):
            data = data.buffer
        elif not isinstance(data, TensorDict):
            raise TypeError("`data` must be a TensorDict or a sheeprl_prey_amd.data.ReplayBuffer")
        if data is None:
            raise RuntimeError("The `data` replay buffer must be not None")
        if len(data.shape) != 2:
            raise RuntimeError(
                "`data` must have 2 batch dimensions: [sequence_length, n_envs]. "
                "`sequence_length` and `n_envs` should be 1. Shape is: {}".format(data.shape)
            )
        data_len = data.shape[0]
        next_pos = (self._pos + data_len) % self._buffer_size
        # wrap-around (also a whole-buffer add landing back on the write head: next_pos == pos)
        if next_pos < self._pos or (data_len >= self._buffer_size and (not self._full or next_pos == self._pos)):
            idxes = torch.cat((torch.arange(self._pos, self._buffer_size), torch.arange(0, next_pos)))
        else:
            idxes = torch.arange(self._pos, next_pos)
        data_to_store = data
        if data_len > self._buffer_size:
            # keep the last `buffer_size` rows, aligned with the wrap-around indices above
            data_to_store = data[data_len - len(idxes) :]
        if len(idxes) > self._buffer_size:
            # never scatter duplicate indices (undefined write order on GPU): keep the newest rows
            idxes = idxes[-self._buffer_size :]
            data_to_store = data_to_store[len(data_to_store) - self._buffer_size :]
        self._ensure_storage(data_to_store)
        dev = self._first_device()
        if dev.type != "cpu" and len(idxes) == next_pos - self._pos > 0:
            # contiguous rows: a slice copy, no index upload.  Device-resident sources of the buffer's dtype
            # (e.g. SAC's one staged row, sliced per key) go as ONE multi-tensor copy launch instead of one
            # copy per key
            dsts, srcs = [], []
            for k, v in data_to_store.items():
                dst = self._buf._data[k][self._pos : next_pos]
                if v.device == dst.device and v.dtype == dst.dtype and v.shape == dst.shape:
                    dsts.append(dst)
                    srcs.append(v)
                    continue
                # pinned / device sources copy without blocking the host (stream-ordered).  A pageable
                # host source must copy synchronously: an async DMA from pageable memory may read it
                # after the caller has freed or overwritten it (seen as NaN gradients once the
                # stream runs a captured train step ahead of the host)
                nb = v.device.type != "cpu" or v.is_pinned()
                dst.copy_(v, non_blocking=nb)
            if len(dsts) > 1:
                torch._foreach_copy_(dsts, srcs)
            elif dsts:
                dsts[0].copy_(srcs[0])
        else:
            idxes = idxes.to(dev)
            for k, v in data_to_store.items():
                dst = self._buf._data[k]
                dst[idxes] = v.to(dst.device, dst.dtype)
        if self._pos + data_len >= self._buffer_size:
            self._full = True
        self._pos = next_pos

    def add_step(self, rows: Dict[str, Tensor]) -> None:
        """Add ONE time step, ``rows[k]`` [n_envs, ...]: ``add`` of the [1, n_envs] TensorDict without building it.
        Device-resident storage fed with device tensors of the stored dtypes and shapes (e.g. SAC's staged
        transition row, sliced per key) takes one multi-tensor copy launch; anything else goes through ``add``."""
        buf = self._buf
        if buf is not None and len(rows) == len(buf._data) and self._first_device().type != "cpu":
            pos = self._pos
            dsts, srcs = [], []
            for k, v in rows.items():
                store = buf._data.get(k)
                if store is None or v.dtype != store.dtype or v.device != store.device or v.shape != store.shape[1:]:
                    break
                dsts.append(store[pos])
                srcs.append(v)
            else:
                torch._foreach_copy_(dsts, srcs)
                self._pos = (pos + 1) % self._buffer_size
                if pos + 1 >= self._buffer_size:
                    self._full = True
                return
        self.add(TensorDict({k: v.unsqueeze(0) for k, v in rows.items()}, batch_size=[1, self._n_envs],
                            device=next(iter(rows.values())).device))

    def _first_device(self):
        for v in self._buf.values():
            return v.device
        return self._device

    # ------------------------------------------------------------------ sample
    def sample(self, batch_size: int, sample_next_obs: bool = False, clone: bool = False, **kwargs) -> TensorDict:
        """Returns a TensorDict of batch ``[batch_size, 1]`` (never the write head)."""
        if batch_size <= 0:
            raise ValueError("Batch size must be greater than 0")
        if not self._full and self._pos == 0:
            raise ValueError("No sample has been added to the buffer. Please add at least one sample calling `self.add()`")
        dev = self._first_device()
        if self._full:
            first_end = self._pos - 1 if sample_next_obs else self._pos
            second_end = self.buffer_size if first_end >= 0 else self.buffer_size + first_end
            n1 = max(first_end, 0)
            n2 = max(second_end - self._pos, 0)
            batch_idxes = _sample_two_ranges(n1, self._pos, n2, batch_size, dev)
        else:
            max_pos = self._pos - 1 if sample_next_obs else self._pos
            if max_pos == 0:
                raise RuntimeError(
                    "You want to sample the next observations, but one sample has been added to the buffer. "
                    "Make sure that at least two samples are added."
                )
            batch_idxes = torch.randint(0, max_pos, size=(batch_size,), device=dev)
        sample = self._get_samples(batch_idxes, sample_next_obs=sample_next_obs).unsqueeze(-1)
        return sample.clone() if clone else sample

    def _get_samples(self, batch_idxes: Tensor, sample_next_obs: bool = False) -> TensorDict:
        if self._buf is None:
            raise RuntimeError("The buffer has not been initialized. Try to add some data first.")
        env_idxes = torch.randint(0, self.n_envs, size=(len(batch_idxes),), device=batch_idxes.device)
        out = self._buf[batch_idxes, env_idxes]
        if sample_next_obs:
            for k in self.obs_keys:
                out.set(f"next_{k}", self._buf[k][(batch_idxes + 1) % self._buffer_size, env_idxes])
        return out

    def sample_rows_into(self, out: Dict[str, Tensor], batch_size: int) -> bool:
        """``sample(batch_size)`` (without next observations) written straight into the preallocated contiguous
        ``out[k]`` [batch_size, ...] - e.g. a captured train step's static inputs - by ONE device launch (rows
        uniform over the filled store, envs uniform: the distribution of ``sample``).  The regular path's index
        draws, per-key gathers and copy-ins become one kernel.  False (nothing written) when not applicable."""
        return self._fused_draw({k: v.unsqueeze(0) for k, v in out.items()}, batch_size, 1)

    def _fused_draw(self, out: Dict[str, Tensor], batch_size: int, sequence_length: int) -> bool:
        """One-launch device draw of ``batch_size`` windows of ``sequence_length`` rows into ``out[k]``
        [sequence_length, batch_size, ...] (``sample_into`` / ``sample_rows_into``)."""
        if self._buf is None or not ops.fused_enabled() or set(out) != set(self._buf.keys()):
            return False
        dev = self._first_device()
        if dev.type != "cuda" or sequence_length < 1:
            return False
        for k, o in out.items():
            # the kernel copies rows verbatim: each destination must have the stored dtype and feature shape
            # (the regular path casts non-uint8 keys to fp32) - otherwise the caller takes the regular path
            b = self._buf[k]
            if (o.dtype != b.dtype or tuple(o.shape) != (sequence_length, batch_size) + tuple(b.shape[2:])
                    or not o.is_contiguous() or o.device != b.device):
                return False
        if not self._full and self._pos - sequence_length + 1 < 1:
            raise ValueError(f"too long sequence length ({sequence_length})")
        if self._full:
            first_end = self._pos - sequence_length + 1
            second_end = self.buffer_size if first_end >= 0 else self.buffer_size + first_end
            n1, start2, n2 = max(first_end, 0), self._pos, max(second_end - self._pos, 0)
        else:
            n1, start2, n2 = self._pos - sequence_length + 1, 0, 0
        if not hasattr(self, "_draw_seed"):
            self._draw_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            self._draw_counter = 0
        keys = list(self._buf.keys())
        self._draw_counter += 1
        return bool(ops._ext().seq_sample_into([self._buf[k] for k in keys], [out[k] for k in keys], int(batch_size),
                                               int(sequence_length), int(n1), int(start2), int(n2), self._draw_seed,
                                               self._draw_counter))

    # ------------------------------------------------------------------ item access
    def __getitem__(self, key: str) -> Tensor:
        if not isinstance(key, str):
            raise TypeError("`key` must be a string")
        if self._buf is None:
            raise RuntimeError("The buffer has not been initialized. Try to add some data first.")
        return self._buf.get(key)

    def __setitem__(self, key: str, t: Tensor) -> None:
        if self._buf is None:
            raise RuntimeError("The buffer has not been initialized. Try to add some data first.")
        if key in self._buf.keys():
            self._buf._data[key].copy_(t)
        else:
            self._buf.set(key, t)

    # ------------------------------------------------------------------ checkpoint
    def state_dict(self) -> Dict:
        buf = {} if self._buf is None else {k: v.detach().cpu().clone() for k, v in self._buf.items()}
        sd = {"buffer": buf, "pos": self._pos, "full": self._full, "buffer_size": self._buffer_size, "n_envs": self._n_envs}
        if hasattr(self, "_draw_seed"):
            # the device-side sampler's stream position: a resumed run continues the index sequence instead of
            # replaying the original run's first draws
            sd["draw_seed"], sd["draw_counter"] = int(self._draw_seed), int(self._draw_counter)
        return sd

    def load_state_dict(self, sd: Dict) -> None:
        if sd["buffer_size"] != self._buffer_size or sd["n_envs"] != self._n_envs:
            raise RuntimeError("replay buffer size mismatch on resume")
        if "draw_seed" in sd:
            self._draw_seed, self._draw_counter = int(sd["draw_seed"]), int(sd["draw_counter"])
        data = TensorDict(sd["buffer"], batch_size=[self._buffer_size, self._n_envs])
        if self._buf is None or len(self._buf.keys()) == 0:
            self._ensure_storage(data)
        for k, v in data.items():
            if k not in self._buf.keys():
                self._ensure_storage(TensorDict({k: v}, batch_size=[self._buffer_size, self._n_envs]))
            self._buf._data[k].copy_(v)
        self._pos = int(sd["pos"])
        self._full = bool(sd["full"])

    def buffers_for_checkpoint(self):
        return [self]


class SequentialReplayBuffer(ReplayBuffer):
    """Samples ``n_samples x batch_size`` sequences of ``sequence_length`` consecutive steps of ONE env."""

    def __init__(self, buffer_size: int, n_envs: int = 1, device="cpu", memmap: bool = False, memmap_dir=None):
        super().__init__(buffer_size, n_envs, device, memmap, memmap_dir)

    def sample(self, batch_size: int, sample_next_obs: bool = False, clone: bool = False, sequence_length: int = 1,
               n_samples: int = 1) -> TensorDict:
        """Returns ``[n_samples, sequence_length, batch_size]``."""
        batch_dim = batch_size * n_samples
        if batch_dim <= 0:
            raise ValueError("Batch size must be greater than 0")
        if not self._full and self._pos == 0:
            raise ValueError("No sample has been added to the buffer. Please add at least one sample calling `self.add()`")
        if self._buf is None:
            raise RuntimeError("The buffer has not been initialized. Try to add some data first.")
        if not self._full and self._pos - sequence_length + 1 < 1:
            raise ValueError(f"too long sequence length ({sequence_length})")
        if self._full and sequence_length > self._buf.shape[0]:
            raise ValueError(f"too long sequence length ({sequence_length})")
        dev = self._first_device()
        if self._full:
            first_end = self._pos - sequence_length + 1
            second_end = self.buffer_size if first_end >= 0 else self.buffer_size + first_end
            n1 = max(first_end, 0)
            n2 = max(second_end - self._pos, 0)
            start_idxes = _sample_two_ranges(n1, self._pos, n2, batch_dim, dev)
        else:
            start_idxes = torch.randint(0, self._pos - sequence_length + 1, size=(batch_dim,), device=dev)
        chunk = torch.arange(sequence_length, device=dev).reshape(1, -1)
        idxes = (start_idxes.reshape(-1, 1) + chunk) % self.buffer_size
        sample = self._get_samples(idxes).reshape(n_samples, batch_size, sequence_length).permute(0, 2, 1)
        return sample.clone() if clone else sample

    def sample_into(self, out: Dict[str, Tensor], batch_size: int, sequence_length: int) -> bool:
        """``sample(batch_size, sequence_length=...)[0]`` written straight into the preallocated contiguous
        ``out[k]`` [sequence_length, batch_size, ...] (e.g. a graphed train step's static inputs) by ONE device
        launch (``gather.hip`` seq_sample_kernel): the start rows and envs are drawn on the device - same
        distribution as ``sample``, a counter-based generator seeded from torch's - so the host does not issue the
        ~15 small ops of the index draw, gather and copy-in.  False (nothing written) when not applicable."""
        return self._fused_draw(out, batch_size, sequence_length)

    def _get_samples(self, batch_idxes: Tensor, sample_next_obs: bool = False) -> TensorDict:
        shape = batch_idxes.shape
        env_idxes = torch.randint(0, self.n_envs, size=(shape[0],), device=batch_idxes.device).view(-1, 1).expand(shape)
        keys = list(self._buf.keys())
        if batch_idxes.is_cuda and 0 < len(keys) <= 16 and ops.fused_enabled() and all(
                self._buf[k].is_cuda and self._buf[k].is_contiguous() for k in keys):
            # every key's sequence rows in one gather launch (ops/csrc/gather.hip); an out-of-range index
            # zero-fills its row and raises the device error word read by ``check_gather_error``
            err = getattr(self, "_gather_err", None)
            if err is None or err.device != batch_idxes.device:
                # word 1 of the device's fault block: the flat optimisers skip the update of a step that set it
                err = self._gather_err = ops.fault_block(batch_idxes.device)[1:2]
            outs = ops._ext().gather_rows([self._buf[k] for k in keys], batch_idxes.reshape(-1).contiguous(),
                                          env_idxes.reshape(-1).contiguous(), err)
            return TensorDict(dict(zip(keys, outs)), batch_size=[batch_idxes.numel()], device=self._buf.device).view(*shape)
        return self._buf[batch_idxes.reshape(-1), env_idxes.reshape(-1)].view(*shape)


    def check_gather_error(self) -> None:
        """Host check of the gather kernel's error word (off the hot path: log / checkpoint time)."""
        err = getattr(self, "_gather_err", None)
        if err is not None and int(err.item()) != 0:
            err.zero_()
            raise RuntimeError("SequentialReplayBuffer: a sampled (row, env) index was outside the store; "
                               "the affected sample rows were zero-filled")


class EpisodeBuffer:
    """Whole episodes; each ends with its only ``done``; FIFO eviction by cumulative length."""

    def __init__(self, buffer_size: int, sequence_length: int, device="cpu", memmap: bool = False, memmap_dir=None) -> None:
        if buffer_size <= 0:
            raise ValueError(f"The buffer size must be greater than zero, got: {buffer_size}")
        if sequence_length <= 0:
            raise ValueError(f"The sequence length must be greater than zero, got: {sequence_length}")
        if buffer_size < sequence_length:
            raise ValueError(
                "The sequence length must be lower than the buffer size, "
                f"got: bs = {buffer_size} and sl = {sequence_length}"
            )
        self._buffer_size = buffer_size
        self._sequence_length = sequence_length
        self._buf: List[TensorDict] = []
        self._cum_lengths: List[int] = []
        self._dirs: List[Optional[Path]] = []
        self._device = torch.device(device) if isinstance(device, str) else device
        self._memmap = memmap
        self._memmap_dir = memmap_dir
        if memmap_dir is None:
            if memmap:
                warnings.warn(
                    "The buffer will be memory-mapped into the `/tmp` folder, this means that there is the"
                    " possibility to lose the saved files. Set the `memmap_dir` to a known directory.",
                    UserWarning,
                )
        else:
            self._memmap_dir = Path(self._memmap_dir)
            self._memmap_dir.mkdir(parents=True, exist_ok=True)
        self._chunk_length = torch.arange(sequence_length).reshape(1, -1)

    @property
    def buffer(self) -> List[TensorDict]:
        return self._buf

    @property
    def buffer_size(self) -> int:
        return self._buffer_size

    @property
    def sequence_length(self) -> int:
        return self._sequence_length

    @property
    def device(self):
        return self._device

    @property
    def is_memmap(self) -> bool:
        return self._memmap

    @property
    def full(self) -> bool:
        return self._cum_lengths[-1] + self._sequence_length > self._buffer_size if len(self._buf) > 0 else False

    @property
    def empty(self) -> bool:
        return len(self._buf) == 0

    def __getitem__(self, key: int) -> TensorDict:
        if not isinstance(key, int):
            raise TypeError("`key` must be an integer")
        return self._buf[key]

    def __len__(self) -> int:
        return self._cum_lengths[-1] if len(self._buf) > 0 else 0

    def _drop_first(self, n: int) -> None:
        for _ in range(n):
            self._buf.pop(0)
            d = self._dirs.pop(0)
            if d is not None and d.exists():
                shutil.rmtree(d, ignore_errors=True)

    def add(self, episode: TensorDict) -> None:
        dones = episode["dones"]
        n_dones = int(torch.count_nonzero(dones).item())
        if n_dones != 1:
            raise RuntimeError(f"The episode must contain exactly one done, got: {n_dones}")
        if float(dones[-1].reshape(-1)[0]) != 1:
            raise RuntimeError(f"The last step must contain a done, got: {dones[-1]}")
        if episode.shape[0] < self._sequence_length:
            raise RuntimeError(f"Episode too short (at least {self._sequence_length} steps), got: {episode.shape[0]} steps")
        if episode.shape[0] > self._buffer_size:
            raise RuntimeError(f"Episode too long (at most {self._buffer_size} steps), got: {episode.shape[0]} steps")
        ep_len = episode.shape[0]
        if self.full or len(self) + ep_len > self._buffer_size:
            cum = np.array(self._cum_lengths)
            mask = (len(self) - cum + ep_len) <= self._buffer_size
            last_to_remove = int(mask.argmax())
            self._drop_first(last_to_remove + 1)
            cum = cum[last_to_remove + 1 :] - cum[last_to_remove]
            self._cum_lengths = cum.tolist()
        self._cum_lengths.append(len(self) + ep_len)
        ep_dir = None
        if self._memmap and self._device.type == "cpu":
            base = self._memmap_dir if self._memmap_dir is not None else Path(os.environ.get("TMPDIR", "/tmp"))
            ep_dir = Path(base) / f"episode_{uuid.uuid4()}"
            ep_dir.mkdir(parents=True, exist_ok=True)
            stored = TensorDict(batch_size=episode.shape, device="cpu")
            for k, v in episode.items():
                t = _alloc(v.shape, v.dtype, "cpu", True, ep_dir / f"{k.replace('/', '_')}.memmap")
                t.copy_(v)
                stored._data[k] = t
            episode = stored
        else:
            episode = episode.to(self._device)
        self._buf.append(episode)
        self._dirs.append(ep_dir)

    def sample(self, batch_size: int, n_samples: int = 1, prioritize_ends: bool = False, clone: bool = False) -> TensorDict:
        """Returns ``[n_samples, sequence_length, batch_size]``."""
        if batch_size <= 0:
            raise ValueError(f"Batch size must be greater than 0, got: {batch_size}")
        if n_samples <= 0:
            raise ValueError(f"The number of samples must be greater than 0, got: {n_samples}")
        if len(self) == 0:
            raise RuntimeError("No sample has been added to the buffer. Please add at least one sample calling `self.add()`")
        per_ep = torch.bincount(torch.randint(0, len(self._buf), (batch_size * n_samples,)))
        samples = []
        for i, n in enumerate(per_ep.tolist()):
            if n == 0:
                continue
            ep_len = self._buf[i].shape[0]
            upper = ep_len - self._sequence_length + 1
            if prioritize_ends:
                upper += self._sequence_length
            start = torch.clamp(torch.randint(0, upper, size=(n,)).reshape(-1, 1), max=ep_len - self._sequence_length)
            samples.append(self._buf[i][start + self._chunk_length])
        out = cat(samples, 0).reshape(n_samples, batch_size, self._sequence_length).permute(0, 2, 1)
        return out.clone() if clone else out

    def state_dict(self) -> Dict:
        return {
            "episodes": [{k: v.detach().cpu().clone() for k, v in ep.items()} for ep in self._buf],
            "buffer_size": self._buffer_size,
            "sequence_length": self._sequence_length,
        }

    def load_state_dict(self, sd: Dict) -> None:
        self._drop_first(len(self._buf))
        self._cum_lengths = []
        for ep in sd["episodes"]:
            n = next(iter(ep.values())).shape[0]
            self.add(TensorDict(ep, batch_size=[n, *next(iter(ep.values())).shape[1:2]]))

    def buffers_for_checkpoint(self):
        return []


class AsyncReplayBuffer:
    """One (Sequential)ReplayBuffer per env so that envs can reset independently."""

    def __init__(self, buffer_size: int, n_envs: int = 1, device="cpu", memmap: bool = False, memmap_dir=None,
                 sequential: bool = False):
        if buffer_size <= 0:
            raise ValueError(f"The buffer size must be greater than zero, got: {buffer_size}")
        if n_envs <= 0:
            raise ValueError(f"The number of environments must be greater than zero, got: {n_envs}")
        self._buffer_size = buffer_size
        self._n_envs = n_envs
        self._device = torch.device(device) if isinstance(device, str) else device
        self._memmap = memmap
        self._memmap_dir = Path(memmap_dir) if memmap_dir is not None else None
        self._sequential = sequential
        self._buf: Optional[List[ReplayBuffer]] = None
        if self._memmap:
            if memmap_dir is None:
                warnings.warn(
                    "The buffer will be memory-mapped into the `/tmp` folder, this means that there is the"
                    " possibility to lose the saved files. Set the `memmap_dir` to a known directory.",
                    UserWarning,
                )
            else:
                self._memmap_dir.mkdir(parents=True, exist_ok=True)

    @property
    def buffer(self):
        return None if self._buf is None else tuple(self._buf)

    @property
    def buffer_size(self) -> int:
        return self._buffer_size

    @property
    def full(self):
        return None if self._buf is None else tuple(b.full for b in self._buf)

    @property
    def n_envs(self) -> int:
        return self._n_envs

    @property
    def shape(self):
        return None if self._buf is None else tuple(b.shape for b in self._buf)

    @property
    def device(self):
        return self._device

    def __len__(self) -> int:
        return self.buffer_size

    def check_gather_error(self) -> None:
        """Raise if any per-env sequential buffer's gather kernel saw an out-of-range index."""
        for b in self._buf or ():
            if isinstance(b, SequentialReplayBuffer):
                b.check_gather_error()

    def _init(self) -> None:
        cls = SequentialReplayBuffer if self._sequential else ReplayBuffer
        self._buf = [
            cls(self.buffer_size, n_envs=1, device=self._device, memmap=self._memmap,
                memmap_dir=(self._memmap_dir / f"env_{i}") if self._memmap_dir is not None else None)
            for i in range(self._n_envs)
        ]

    def add(self, data: TensorDict, indices: Optional[Sequence[int]] = None) -> None:
        if not isinstance(data, TensorDict):
            raise TypeError("`data` must be a TensorDict")
        if len(data.shape) != 2:
            raise RuntimeError(
                "`data` must have 2 batch dimensions: [sequence_length, n_envs]. "
                "`sequence_length` and `n_envs` should be 1. Shape is: {}".format(data.shape)
            )
        if self._buf is None:
            self._init()
        if indices is None:
            indices = tuple(range(self.n_envs))
        for j, env_idx in enumerate(indices):
            self._buf[env_idx].add(data[:, j : j + 1])

    def sample(self, batch_size: int, sample_next_obs: bool = False, clone: bool = False, sequence_length: int = 1,
               n_samples: int = 1) -> TensorDict:
        if batch_size <= 0 or n_samples <= 0:
            raise ValueError(f"`batch_size` ({batch_size}) and `n_samples` ({n_samples}) must be both greater than 0")
        if self._buf is None:
            raise RuntimeError("The buffer has not been initialized. Try to add some data first.")
        if self._n_envs == 1:
            per_buf = [batch_size]
        else:
            per_buf = torch.bincount(torch.randint(0, self._n_envs, (batch_size,)), minlength=self._n_envs).tolist()
        samples = [
            b.sample(batch_size=bs, sample_next_obs=sample_next_obs, clone=clone, n_samples=n_samples,
                     sequence_length=sequence_length)
            for b, bs in zip(self._buf, per_buf)
            if bs > 0
        ]
        if len(samples) == 1:  # one env buffer drew everything: no concatenation copy
            return samples[0]
        return cat(samples, dim=2 if self._sequential else 0)

    def sample_into(self, out: Dict[str, Tensor], batch_size: int, sequence_length: int) -> bool:
        """One env buffer: its fused device-side sample into ``out`` (``SequentialReplayBuffer.sample_into``)."""
        if self._buf is None or self._n_envs != 1 or not self._sequential:
            return False
        return self._buf[0].sample_into(out, batch_size, sequence_length)

    def state_dict(self) -> Dict:
        return {"buffers": [] if self._buf is None else [b.state_dict() for b in self._buf], "n_envs": self._n_envs,
                "buffer_size": self._buffer_size, "sequential": self._sequential}

    def load_state_dict(self, sd: Dict) -> None:
        if sd["n_envs"] != self._n_envs:
            raise RuntimeError(f"Given {sd['n_envs']} env buffers, but {self._n_envs} envs are instantiated")
        if not sd["buffers"]:
            return
        self._init()
        for b, s in zip(self._buf, sd["buffers"]):
            b.load_state_dict(s)

    def buffers_for_checkpoint(self):
        return [] if self._buf is None else list(self._buf)
