"""Audio datasets (reference: python/paddle/audio/datasets/{esc50,tess}.py).

The reference downloads the archives; here there is no network, so a dataset reads an already
extracted copy from ``data_dir`` (same directory layout as the official archive) and raises a
clear error when it is absent.
"""
from __future__ import annotations

import os

from ...io import Dataset


class AudioClassificationDataset(Dataset):
    def __init__(self, files, labels, feat_type="raw", sample_rate=None, **kwargs):
        self.files, self.labels, self.feat_type = files, labels, feat_type
        self.sample_rate = sample_rate
        self.feat_config = kwargs

    def _convert(self, waveform, sr):
        from .. import features

        if self.feat_type == "raw":
            return waveform
        layer = {"melspectrogram": features.MelSpectrogram, "logmelspectrogram": features.LogMelSpectrogram,
                 "mfcc": features.MFCC, "spectrogram": features.Spectrogram}[self.feat_type.lower()]
        kw = dict(self.feat_config)
        if self.feat_type.lower() != "spectrogram":
            kw.setdefault("sr", sr)
        return layer(**kw)(waveform.unsqueeze(0)).squeeze(0)

    def __getitem__(self, idx):
        from ..backends import load

        wav, sr = load(self.files[idx])
        return self._convert(wav[0], sr), self.labels[idx]

    def __len__(self):
        return len(self.files)


def _need(path, name):
    if not path or not os.path.isdir(path):
        raise FileNotFoundError(f"{name}: pass data_dir= pointing at the extracted dataset (no download offline)")


class ESC50(AudioClassificationDataset):
    """ESC-50: 2000 5-second clips, 50 classes, 5 folds (meta/esc50.csv)."""

    def __init__(self, mode="train", split=1, feat_type="raw", data_dir=None, **kwargs):
        _need(data_dir, "ESC50")
        import csv

        files, labels = [], []
        with open(os.path.join(data_dir, "meta", "esc50.csv")) as f:
            for row in csv.DictReader(f):
                fold = int(row["fold"])
                if (mode == "train") == (fold != split):
                    files.append(os.path.join(data_dir, "audio", row["filename"]))
                    labels.append(int(row["target"]))
        super().__init__(files, labels, feat_type, **kwargs)


class TESS(AudioClassificationDataset):
    """Toronto emotional speech set: labels are the emotion suffix of each wav file name."""

    label_list = ["angry", "disgust", "fear", "happy", "neutral", "ps", "sad"]

    def __init__(self, mode="train", n_folds=5, split=1, feat_type="raw", data_dir=None, **kwargs):
        _need(data_dir, "TESS")
        wavs = sorted(os.path.join(r, f) for r, _, fs in os.walk(data_dir) for f in fs if f.endswith(".wav"))
        files, labels = [], []
        for i, p in enumerate(wavs):
            fold = i % n_folds + 1
            if (mode == "train") == (fold != split):
                emo = os.path.splitext(os.path.basename(p))[0].split("_")[-1].lower()
                files.append(p)
                labels.append(self.label_list.index(emo))
        super().__init__(files, labels, feat_type, **kwargs)
