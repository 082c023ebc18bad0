"""paddle.signal (reference: python/paddle/signal.py)."""
import torch as _t

from .framework.tensor import Tensor

_w = Tensor._wrap


def stft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, pad_mode="reflect", normalized=False,
         onesided=True, name=None):
    return _w(_t.stft(x._t, n_fft, hop_length, win_length, None if window is None else window._t, center, pad_mode,
                      normalized, onesided, return_complex=True))


def istft(x, n_fft, hop_length=None, win_length=None, window=None, center=True, normalized=False, onesided=True,
          length=None, return_complex=False, name=None):
    return _w(_t.istft(x._t, n_fft, hop_length, win_length, None if window is None else window._t, center, normalized,
                       onesided, length, return_complex))


def frame(x, frame_length, hop_length, axis=-1, name=None):
    return _w(x._t.unfold(axis, frame_length, hop_length).movedim(-1, axis if axis >= 0 else axis - 1))


def overlap_add(x, hop_length, axis=-1, name=None):
    t = x._t
    fl, nf = t.shape[-2], t.shape[-1]
    out = _t.zeros(t.shape[:-2] + ((nf - 1) * hop_length + fl,), dtype=t.dtype, device=t.device)
    for i in range(nf):
        out[..., i * hop_length:i * hop_length + fl] += t[..., i]
    return _w(out)
