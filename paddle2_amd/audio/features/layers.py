"""Audio feature layers (reference: python/paddle/audio/features/layers.py — Spectrogram :86,
MelSpectrogram :178, LogMelSpectrogram :285, MFCC :391).  Input ``(N, T)`` waveforms; outputs
``(N, bins, frames)``."""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor
from ...nn.layer.layers import Layer
from ..functional import compute_fbank_matrix, create_dct, get_window, power_to_db


class Spectrogram(Layer):
    def __init__(self, n_fft=512, hop_length=512, win_length=None, window="hann", power=1.0, center=True,
                 pad_mode="reflect", dtype="float32"):
        super().__init__()
        assert power > 0, "power of spectrogram must be > 0"
        self.n_fft, self.power = n_fft, power
        self.win_length = win_length or n_fft
        self.hop_length = hop_length if hop_length is not None else self.win_length // 4
        self.center, self.pad_mode = center, pad_mode
        self.register_buffer("fft_window", get_window(window, self.win_length, fftbins=True, dtype=dtype),
                             persistable=False)

    def forward(self, x):
        t = x._t if isinstance(x, Tensor) else torch.as_tensor(x)
        win = self.fft_window._t.to(t.device)
        spec = torch.stft(t, self.n_fft, self.hop_length, self.win_length, win.to(t.dtype), self.center,
                          self.pad_mode, False, True, return_complex=True)
        return Tensor._wrap(spec.abs().pow(self.power))


class MelSpectrogram(Layer):
    def __init__(self, sr=22050, n_fft=2048, hop_length=512, win_length=None, window="hann", power=2.0,
                 center=True, pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None, htk=False, norm="slaney",
                 dtype="float32"):
        super().__init__()
        self._spectrogram = Spectrogram(n_fft, hop_length, win_length, window, power, center, pad_mode, dtype)
        self.n_mels, self.f_min, self.f_max, self.htk, self.norm = n_mels, f_min, f_max, htk, norm
        f_max = f_max if f_max is not None else sr // 2
        self.register_buffer("fbank_matrix", compute_fbank_matrix(sr, n_fft, n_mels, f_min, f_max, htk, norm, dtype),
                             persistable=False)

    def forward(self, x):
        spec = self._spectrogram(x)._t
        fb = self.fbank_matrix._t.to(spec.device, spec.dtype)
        return Tensor._wrap(torch.matmul(fb, spec))


class LogMelSpectrogram(Layer):
    def __init__(self, sr=22050, n_fft=512, hop_length=None, win_length=None, window="hann", power=2.0,
                 center=True, pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None, htk=False, norm="slaney",
                 ref_value=1.0, amin=1e-10, top_db=None, dtype="float32"):
        super().__init__()
        self._melspectrogram = MelSpectrogram(sr, n_fft, hop_length, win_length, window, power, center, pad_mode,
                                              n_mels, f_min, f_max, htk, norm, dtype)
        self.ref_value, self.amin, self.top_db = ref_value, amin, top_db

    def forward(self, x):
        return power_to_db(self._melspectrogram(x), self.ref_value, self.amin, self.top_db)


class MFCC(Layer):
    def __init__(self, sr=22050, n_mfcc=40, n_fft=512, hop_length=None, win_length=None, window="hann", power=2.0,
                 center=True, pad_mode="reflect", n_mels=64, f_min=50.0, f_max=None, htk=False, norm="slaney",
                 ref_value=1.0, amin=1e-10, top_db=None, dtype="float32"):
        super().__init__()
        assert n_mfcc <= n_mels, f"n_mfcc ({n_mfcc}) must not exceed n_mels ({n_mels})"
        self._log_melspectrogram = LogMelSpectrogram(sr, n_fft, hop_length, win_length, window, power, center,
                                                     pad_mode, n_mels, f_min, f_max, htk, norm, ref_value, amin,
                                                     top_db, dtype)
        self.register_buffer("dct_matrix", create_dct(n_mfcc, n_mels, dtype=dtype), persistable=False)

    def forward(self, x):
        lm = self._log_melspectrogram(x)._t
        d = self.dct_matrix._t.to(lm.device, lm.dtype)
        return Tensor._wrap(torch.matmul(lm.transpose(1, 2), d).transpose(1, 2))
