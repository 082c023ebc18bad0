from .layers import MFCC, LogMelSpectrogram, MelSpectrogram, Spectrogram  # noqa: F401

__all__ = ["Spectrogram", "MelSpectrogram", "LogMelSpectrogram", "MFCC"]
