"""Audio I/O (reference: python/paddle/audio/backends/wave_backend.py, init_backend.py).

The built-in backend reads/writes PCM WAV with the standard-library ``wave`` module (the
reference's default "wave_backend"); ``soundfile`` is used when importable.
"""
from __future__ import annotations

import wave as _wave

import numpy as np
import torch

from ...framework.tensor import Tensor

_backend = ["wave_backend"]


class AudioInfo:
    def __init__(self, sample_rate, num_samples, num_channels, bits_per_sample, encoding):
        self.sample_rate, self.num_frames, self.num_channels = sample_rate, num_samples, num_channels
        self.bits_per_sample, self.encoding = bits_per_sample, encoding


def list_available_backends():
    out = ["wave_backend"]
    try:
        import soundfile  # noqa: F401

        out.append("soundfile")
    except ImportError:
        pass
    return out


def get_current_backend():
    return _backend[0]


def set_backend(name):
    if name not in list_available_backends():
        raise NotImplementedError(f"audio backend {name!r} is not available")
    _backend[0] = name


def info(filepath):
    with _wave.open(str(filepath), "rb") as f:
        return AudioInfo(f.getframerate(), f.getnframes(), f.getnchannels(), f.getsampwidth() * 8, "PCM_S")


_DT = {1: np.uint8, 2: np.int16, 4: np.int32}


def load(filepath, frame_offset=0, num_frames=-1, normalize=True, channels_first=True):
    """-> (waveform Tensor [C, T] (or [T, C]), sample_rate)."""
    with _wave.open(str(filepath), "rb") as f:
        sr, ch, sw = f.getframerate(), f.getnchannels(), f.getsampwidth()
        f.setpos(frame_offset)
        n = f.getnframes() - frame_offset if num_frames < 0 else num_frames
        raw = f.readframes(n)
    a = np.frombuffer(raw, dtype=_DT[sw]).reshape(-1, ch)
    if normalize:
        if sw == 1:
            a = (a.astype(np.float32) - 128.0) / 128.0
        else:
            a = a.astype(np.float32) / float(2 ** (8 * sw - 1))
    t = torch.from_numpy(np.ascontiguousarray(a.T if channels_first else a))
    return Tensor._wrap(t), sr


def save(filepath, src, sample_rate, channels_first=True, encoding=None, bits_per_sample=16):
    x = src._t if isinstance(src, Tensor) else torch.as_tensor(src)
    a = x.detach().cpu().numpy()
    if a.ndim == 1:
        a = a[None]
    if channels_first:
        a = a.T
    if a.dtype.kind == "f":
        a = np.clip(a, -1.0, 1.0 - 1.0 / 32768) * 32768.0
    a = a.astype(np.int16)
    with _wave.open(str(filepath), "wb") as f:
        f.setnchannels(a.shape[1])
        f.setsampwidth(2)
        f.setframerate(int(sample_rate))
        f.writeframes(a.tobytes())
