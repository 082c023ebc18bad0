from .functional import (compute_fbank_matrix, create_dct, fft_frequencies, hz_to_mel, mel_frequencies,  # noqa: F401
                         mel_to_hz, power_to_db)
from .window import get_window  # noqa: F401

__all__ = ["compute_fbank_matrix", "create_dct", "fft_frequencies", "hz_to_mel", "mel_frequencies", "mel_to_hz",
           "power_to_db", "get_window"]
