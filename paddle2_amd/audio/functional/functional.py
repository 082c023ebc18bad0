"""Mel-scale helpers (reference: python/paddle/audio/functional/functional.py:29 hz_to_mel,
:83 mel_to_hz, :126 mel_frequencies, :166 fft_frequencies, :189 compute_fbank_matrix,
:262 power_to_db, :306 create_dct).  Slaney (default) and HTK mel scales, librosa conventions."""
from __future__ import annotations

import math

import torch

from ...framework.dtype import convert_dtype
from ...framework.tensor import Tensor

_w = Tensor._wrap

# Slaney scale: linear below 1 kHz (200/3 Hz per mel), logarithmic above
_F_SP = 200.0 / 3
_MIN_LOG_HZ = 1000.0
_MIN_LOG_MEL = _MIN_LOG_HZ / _F_SP
_LOGSTEP = math.log(6.4) / 27.0


def hz_to_mel(freq, htk=False):
    if isinstance(freq, Tensor):
        f = freq._t
        if htk:
            return _w(2595.0 * torch.log10(1.0 + f / 700.0))
        lin = f / _F_SP
        log = _MIN_LOG_MEL + torch.log(f / _MIN_LOG_HZ + 1e-10) / _LOGSTEP
        return _w(torch.where(f > _MIN_LOG_HZ, log, lin))
    if htk:
        return 2595.0 * math.log10(1.0 + freq / 700.0)
    if freq >= _MIN_LOG_HZ:
        return _MIN_LOG_MEL + math.log(freq / _MIN_LOG_HZ + 1e-10) / _LOGSTEP
    return freq / _F_SP


def mel_to_hz(mel, htk=False):
    if isinstance(mel, Tensor):
        m = mel._t
        if htk:
            return _w(700.0 * (10.0 ** (m / 2595.0) - 1.0))
        lin = _F_SP * m
        log = _MIN_LOG_HZ * torch.exp(_LOGSTEP * (m - _MIN_LOG_MEL))
        return _w(torch.where(m > _MIN_LOG_MEL, log, lin))
    if htk:
        return 700.0 * (10.0 ** (mel / 2595.0) - 1.0)
    if mel >= _MIN_LOG_MEL:
        return _MIN_LOG_HZ * math.exp(_LOGSTEP * (mel - _MIN_LOG_MEL))
    return _F_SP * mel


def mel_frequencies(n_mels=64, f_min=0.0, f_max=11025.0, htk=False, dtype="float32"):
    lo, hi = hz_to_mel(f_min, htk), hz_to_mel(f_max, htk)
    mels = Tensor._wrap(torch.linspace(lo, hi, n_mels, dtype=torch.float64))
    return _w(mel_to_hz(mels, htk)._t.to(convert_dtype(dtype)))


def fft_frequencies(sr, n_fft, dtype="float32"):
    return _w(torch.linspace(0, float(sr) / 2, int(1 + n_fft // 2), dtype=torch.float64).to(convert_dtype(dtype)))


def compute_fbank_matrix(sr, n_fft, n_mels=64, f_min=0.0, f_max=None, htk=False, norm="slaney", dtype="float32"):
    """Triangular mel filter bank, shape ``(n_mels, n_fft//2 + 1)``."""
    f_max = float(sr) / 2 if f_max is None else f_max
    fftf = fft_frequencies(sr, n_fft, "float64")._t
    melf = mel_frequencies(n_mels + 2, f_min, f_max, htk, "float64")._t
    fdiff = melf[1:] - melf[:-1]
    ramps = melf[:, None] - fftf[None, :]
    lower = -ramps[:n_mels] / fdiff[:n_mels, None]
    upper = ramps[2:n_mels + 2] / fdiff[1:n_mels + 1, None]
    w = torch.clamp(torch.minimum(lower, upper), min=0.0)
    if norm == "slaney":
        w = w * (2.0 / (melf[2:n_mels + 2] - melf[:n_mels]))[:, None]
    elif isinstance(norm, (int, float)):
        w = torch.nn.functional.normalize(w, p=norm, dim=-1)
    return _w(w.to(convert_dtype(dtype)))


def power_to_db(spect, ref_value=1.0, amin=1e-10, top_db=80.0):
    if amin <= 0:
        raise ValueError("amin must be strictly positive")
    if ref_value <= 0:
        raise ValueError("ref_value must be strictly positive")
    s = spect._t if isinstance(spect, Tensor) else torch.as_tensor(spect)
    out = 10.0 * torch.log10(torch.clamp(s, min=amin)) - 10.0 * math.log10(max(ref_value, amin))
    if top_db is not None:
        if top_db < 0:
            raise ValueError("top_db must be non-negative")
        out = torch.maximum(out, out.max() - top_db)
    return _w(out)


def create_dct(n_mfcc, n_mels, norm="ortho", dtype="float32"):
    """DCT-II basis, shape ``(n_mels, n_mfcc)`` (so ``mfcc = log_mel^T @ dct``)."""
    n = torch.arange(n_mels, dtype=torch.float64)
    k = torch.arange(n_mfcc, dtype=torch.float64)
    dct = torch.cos(math.pi / n_mels * (n[:, None] + 0.5) * k[None, :])
    if norm is None:
        dct = dct * 2.0
    else:
        assert norm == "ortho"
        dct[:, 0] *= 1.0 / math.sqrt(2.0)
        dct *= math.sqrt(2.0 / n_mels)
    return _w(dct.to(convert_dtype(dtype)))
