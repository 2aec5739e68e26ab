"""Rank-0 metric logging with a native TensorBoard event-file writer.

The reference logs through Lightning's ``TensorBoardLogger`` (``sheeprl/utils/logger.py:11-39``),
which needs the ``tensorboard`` package - absent from the MI355X image.  TensorBoard's
on-disk format is just TFRecord-framed ``Event`` protobufs, so we write it directly:
``[len:u64][masked_crc32c(len):u32][event bytes][masked_crc32c(event):u32]`` with the
``Event{wall_time=1, step=2, file_version=3, summary=5{value=1{tag=1, simple_value=2}}}``
fields hand-encoded.  The same scalars are mirrored to ``metrics.jsonl`` for scripts.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import time
from typing import Any, Dict, Optional, Tuple

import yaml

# ---------------------------------------------------------------- crc32c (Castagnoli)
_CRC_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ 0x82F63B78 if _c & 1 else _c >> 1
    _CRC_TABLE.append(_c)


def crc32c(data: bytes) -> int:
    crc = 0xFFFFFFFF
    tbl = _CRC_TABLE
    for b in data:
        crc = tbl[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc32c(data: bytes) -> int:
    crc = crc32c(data)
    return (((crc >> 15) | (crc << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---------------------------------------------------------------- protobuf encoding
def _varint(n: int) -> bytes:
    out = bytearray()
    n &= (1 << 64) - 1
    while True:
        b = n & 0x7F
        n >>= 7
        if n:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wire: int) -> bytes:
    return _varint((field << 3) | wire)


def _len_delim(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def encode_scalar_event(tag: str, value: float, step: int, wall_time: Optional[float] = None) -> bytes:
    val = _len_delim(1, tag.encode("utf-8")) + _key(2, 5) + struct.pack("<f", float(value))
    summary = _len_delim(1, val)
    ev = _key(1, 1) + struct.pack("<d", wall_time or time.time()) + _key(2, 0) + _varint(int(step)) + _len_delim(5, summary)
    return ev


def encode_version_event() -> bytes:
    return _key(1, 1) + struct.pack("<d", time.time()) + _len_delim(3, b"brain.Event:2")


def frame_record(data: bytes) -> bytes:
    header = struct.pack("<Q", len(data))
    return header + struct.pack("<I", masked_crc32c(header)) + data + struct.pack("<I", masked_crc32c(data))


def read_events(path: str):
    """Parse an event file written by :class:`EventFileWriter` -> list of (tag, value, step)."""
    out = []
    with open(path, "rb") as f:
        buf = f.read()
    i = 0
    while i + 12 <= len(buf):
        (n,) = struct.unpack("<Q", buf[i : i + 8])
        data = buf[i + 12 : i + 12 + n]
        i += 12 + n + 4
        j, step, summ = 0, 0, None
        while j < len(data):
            k = data[j]
            j += 1
            field, wire = k >> 3, k & 7
            if wire == 1:
                j += 8
            elif wire == 0:
                v, shift = 0, 0
                while True:
                    b = data[j]
                    j += 1
                    v |= (b & 0x7F) << shift
                    shift += 7
                    if not b & 0x80:
                        break
                if field == 2:
                    step = v
            elif wire == 2:
                ln, shift = 0, 0
                while True:
                    b = data[j]
                    j += 1
                    ln |= (b & 0x7F) << shift
                    shift += 7
                    if not b & 0x80:
                        break
                if field == 5:
                    summ = data[j : j + ln]
                j += ln
        if summ is not None:
            # summary -> value(1) -> tag(1), simple_value(2)
            val = summ[2:] if summ[1] < 128 else summ[3:]
            tl = val[1]
            tag = val[2 : 2 + tl].decode()
            (fv,) = struct.unpack("<f", val[2 + tl + 1 : 2 + tl + 5])
            out.append((tag, fv, step))
    return out


class EventFileWriter:
    def __init__(self, log_dir: str):
        os.makedirs(log_dir, exist_ok=True)
        fname = f"events.out.tfevents.{int(time.time())}.{socket.gethostname()}.{os.getpid()}.0"
        self.path = os.path.join(log_dir, fname)
        self._f = open(self.path, "ab")
        self._f.write(frame_record(encode_version_event()))
        self._f.flush()

    def add_scalar(self, tag: str, value: float, step: int) -> None:
        self._f.write(frame_record(encode_scalar_event(tag, value, step)))

    def flush(self) -> None:
        self._f.flush()

    def close(self) -> None:
        if not self._f.closed:
            self._f.flush()
            self._f.close()


class TensorBoardLogger:
    """``root_dir/name/version_<k>`` layout, like Lightning's logger (reference ``logger.py:21-29``)."""

    def __init__(self, root_dir: str, name: str = "", version: Optional[int] = None):
        self.root_dir = root_dir
        self.name = name
        base = os.path.join(root_dir, name) if name else root_dir
        if version is None:
            version = 0
            if os.path.isdir(base):
                existing = [d for d in os.listdir(base) if d.startswith("version_") and d[8:].isdigit()]
                if existing:
                    version = max(int(d[8:]) for d in existing) + 1
        self.version = version
        self.log_dir = os.path.join(base, f"version_{version}")
        os.makedirs(self.log_dir, exist_ok=True)
        self._writer: Optional[EventFileWriter] = None
        self._jsonl = None

    @property
    def writer(self) -> EventFileWriter:
        if self._writer is None:
            self._writer = EventFileWriter(self.log_dir)
            self._jsonl = open(os.path.join(self.log_dir, "metrics.jsonl"), "a")
        return self._writer

    def log_metrics(self, metrics: Dict[str, Any], step: int) -> None:
        w = self.writer
        rec = {"step": int(step)}
        for k, v in metrics.items():
            try:
                fv = float(v)
            except (TypeError, ValueError):
                continue
            w.add_scalar(k, fv, step)
            rec[k] = fv
        self._jsonl.write(json.dumps(rec) + "\n")
        self._jsonl.flush()
        w.flush()

    def log_hyperparams(self, params: Dict[str, Any]) -> None:
        from sheeprl_prey_amd.utils.utils import dotdict

        plain = dotdict(params).as_dict() if isinstance(params, dict) else params
        with open(os.path.join(self.log_dir, "hparams.yaml"), "w") as f:
            yaml.safe_dump(plain, f, sort_keys=False)

    def finalize(self, *_args) -> None:
        if self._writer is not None:
            self._writer.close()
        if self._jsonl is not None:
            self._jsonl.close()


def create_tensorboard_logger(runner, cfg: Dict[str, Any]) -> Tuple[Optional[TensorBoardLogger], str]:
    """Rank 0 creates the logger and broadcasts its ``log_dir`` (reference ``logger.py:11-39``)."""
    root_dir = os.path.join("logs", "runs", cfg.root_dir)
    if runner.is_global_zero:
        logger = TensorBoardLogger(root_dir=root_dir, name=cfg.run_name)
        log_dir = logger.log_dir
    else:
        logger, log_dir = None, None
    log_dir = runner.broadcast_object(log_dir, src=0)
    return logger, log_dir
