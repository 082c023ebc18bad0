"""paddle.fft (reference: python/paddle/fft.py) on rocFFT through ATen."""
import torch as _t

from .framework.tensor import Tensor

_w = Tensor._wrap


def _mk(fn):
    def op(x, n=None, axis=-1, norm="backward", name=None):
        return _w(fn(x._t, n=n, dim=axis, norm=norm))
    return op


def _mkn(fn):
    def op(x, s=None, axes=None, norm="backward", name=None):
        return _w(fn(x._t, s=s, dim=axes, norm=norm))
    return op


fft, ifft, rfft, irfft, hfft, ihfft = (_mk(f) for f in (_t.fft.fft, _t.fft.ifft, _t.fft.rfft, _t.fft.irfft,
                                                         _t.fft.hfft, _t.fft.ihfft))
fftn, ifftn, rfftn, irfftn = (_mkn(f) for f in (_t.fft.fftn, _t.fft.ifftn, _t.fft.rfftn, _t.fft.irfftn))


def fft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return _w(_t.fft.fft2(x._t, s=s, dim=axes, norm=norm))


def ifft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return _w(_t.fft.ifft2(x._t, s=s, dim=axes, norm=norm))


def rfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return _w(_t.fft.rfft2(x._t, s=s, dim=axes, norm=norm))


def irfft2(x, s=None, axes=(-2, -1), norm="backward", name=None):
    return _w(_t.fft.irfft2(x._t, s=s, dim=axes, norm=norm))


def fftfreq(n, d=1.0, dtype=None, name=None):
    return _w(_t.fft.fftfreq(n, d))


def rfftfreq(n, d=1.0, dtype=None, name=None):
    return _w(_t.fft.rfftfreq(n, d))


def fftshift(x, axes=None, name=None):
    return _w(_t.fft.fftshift(x._t, dim=axes))


def ifftshift(x, axes=None, name=None):
    return _w(_t.fft.ifftshift(x._t, dim=axes))
