"""paddle.audio (reference: python/paddle/audio/ — features/layers.py, functional/functional.py,
functional/window.py, backends/wave_backend.py, datasets/{esc50,tess}.py).

Feature extraction runs on the device the waveform lives on: the STFT is ``torch.stft`` (rocFFT on
the MI355X), the mel projection and DCT are GEMMs.
"""
from . import backends, datasets, features, functional  # noqa: F401
from .backends import info, load, save  # noqa: F401

__all__ = ["functional", "features", "datasets", "backends", "load", "info", "save"]
