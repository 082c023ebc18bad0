"""Text datasets (reference: python/paddle/text/datasets/{uci_housing,imdb,imikolov,movielens,
conll05,wmt14,wmt16}.py).

There is no network here: every dataset reads a local copy of the official archive via
``data_file=`` (the reference's download cache path) and raises a clear error when it is missing.
UCIHousing, Imdb, Imikolov and Movielens parse their archives; Conll05st / WMT14 / WMT16 read the
pre-tokenised archives' line formats.
"""
from __future__ import annotations

import collections
import os
import re
import tarfile
import zipfile

import numpy as np

from ..io import Dataset


def _need(path, name):
    if path is None or not os.path.exists(path):
        raise FileNotFoundError(f"{name}: pass data_file= pointing at a local copy of the archive "
                                "(datasets cannot be downloaded offline)")


class UCIHousing(Dataset):
    """Boston housing: 13 features (mean-centred, range-scaled) + price; 80/20 train/test split."""

    def __init__(self, data_file=None, mode="train", download=True):
        assert mode in ("train", "test")
        _need(data_file, "UCIHousing")
        self.mode, self.dtype = mode, "float32"
        data = np.fromfile(data_file, sep=" ").reshape(-1, 14)
        hi, lo, mean = data.max(0), data.min(0), data.mean(0)
        data[:, :13] = (data[:, :13] - mean[:13]) / (hi[:13] - lo[:13])
        cut = int(data.shape[0] * 0.8)
        self.data = data[:cut] if mode == "train" else data[cut:]

    def __getitem__(self, idx):
        row = self.data[idx]
        return row[:-1].astype(self.dtype), row[-1:].astype(self.dtype)

    def __len__(self):
        return len(self.data)


def _tokens(text):
    return text.rstrip("\n\r").translate(str.maketrans("", "", "!\"#$%&'()*+,-./:;<=>?@[\\]^_`{|}~")).lower().split()


class Imdb(Dataset):
    """aclImdb sentiment: (word ids, label) with label 0 = pos, 1 = neg; vocabulary = words seen more
    than ``cutoff`` times in train+test, plus ``<unk>``."""

    def __init__(self, data_file=None, mode="train", cutoff=150, download=True):
        assert mode in ("train", "test")
        _need(data_file, "Imdb")
        self.data_file, self.mode = data_file, mode
        self.word_idx = self._vocab(cutoff)
        unk = self.word_idx["<unk>"]
        self.docs, self.labels = [], []
        for lab, pol in ((0, "pos"), (1, "neg")):
            for doc in self._docs(re.compile(rf"aclImdb/{mode}/{pol}/.*\.txt$")):
                self.docs.append([self.word_idx.get(w, unk) for w in doc])
                self.labels.append(lab)

    def _docs(self, pattern):
        with tarfile.open(self.data_file) as tf:
            for m in tf:
                if pattern.match(m.name):
                    yield _tokens(tf.extractfile(m).read().decode("latin-1"))

    def _vocab(self, cutoff):
        freq = collections.Counter()
        for doc in self._docs(re.compile(r"aclImdb/((train)|(test))/((pos)|(neg))/.*\.txt$")):
            freq.update(doc)
        words = sorted(((w, c) for w, c in freq.items() if c > cutoff), key=lambda x: (-x[1], x[0]))
        idx = {w: i for i, (w, _) in enumerate(words)}
        idx["<unk>"] = len(words)
        return idx

    def __getitem__(self, idx):
        return np.array(self.docs[idx]), np.array([self.labels[idx]])

    def __len__(self):
        return len(self.docs)


class Imikolov(Dataset):
    """PTB language model (simple-examples): 'NGRAM' windows of ``window_size`` ids or 'SEQ'
    (src, trg) pairs; vocabulary = train words with frequency > ``min_word_freq``."""

    def __init__(self, data_file=None, data_type="NGRAM", window_size=-1, mode="train", min_word_freq=50,
                 download=True):
        assert data_type.upper() in ("NGRAM", "SEQ") and mode in ("train", "test")
        _need(data_file, "Imikolov")
        self.data_type, self.window_size = data_type.upper(), window_size
        name = "./simple-examples/data/ptb.{}.txt"
        with tarfile.open(data_file) as tf:
            train = tf.extractfile(name.format("train")).read().decode().splitlines()
            lines = train if mode == "train" else tf.extractfile(name.format("valid")).read().decode().splitlines()
        freq = collections.Counter()
        for ln in train:
            freq.update(ln.strip().split())
            freq.update(["<s>", "<e>"])
        freq.pop("<unk>", None)
        words = sorted(((w, c) for w, c in freq.items() if c > min_word_freq), key=lambda x: (-x[1], x[0]))
        self.word_idx = {w: i for i, (w, _) in enumerate(words)}
        self.word_idx["<unk>"] = len(words)
        unk = self.word_idx["<unk>"]
        self.data = []
        for ln in lines:
            if self.data_type == "NGRAM":
                assert window_size > -1, "NGRAM needs window_size"
                ids = [self.word_idx.get(w, unk) for w in ["<s>"] + ln.strip().split() + ["<e>"]]
                for i in range(window_size, len(ids) + 1):
                    self.data.append(tuple(ids[i - window_size:i]))
            else:
                ids = [self.word_idx.get(w, unk) for w in ln.strip().split()]
                src = [self.word_idx["<s>"]] + ids
                trg = ids + [self.word_idx["<e>"]]
                if window_size > 0 and len(src) > window_size:
                    continue
                self.data.append((src, trg))

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


class Movielens(Dataset):
    """MovieLens-1M ratings joined with user/movie features; deterministic train/test split by
    ``rand_seed`` and ``test_ratio``."""

    def __init__(self, data_file=None, mode="train", test_ratio=0.1, rand_seed=0, download=True):
        assert mode in ("train", "test")
        _need(data_file, "Movielens")
        rng = np.random.default_rng(rand_seed)
        with zipfile.ZipFile(data_file) as z:
            read = lambda n: z.read(f"ml-1m/{n}").decode("latin-1").splitlines()  # noqa: E731
            movies, users = {}, {}
            cats, titles = {}, {}
            for ln in read("movies.dat"):
                mid, title, genres = ln.strip().split("::")
                title = re.sub(r"\(\d{4}\)$", "", title).strip().lower()
                gids = [cats.setdefault(g, len(cats)) for g in genres.split("|")]
                tids = [titles.setdefault(w, len(titles)) for w in title.split()]
                movies[int(mid)] = (gids, tids)
            ages = [1, 18, 25, 35, 45, 50, 56]
            for ln in read("users.dat"):
                uid, gender, age, job, _ = ln.strip().split("::")
                users[int(uid)] = (0 if gender == "M" else 1, ages.index(int(age)), int(job))
            self.data = []
            for ln in read("ratings.dat"):
                if (rng.random() < test_ratio) == (mode == "test"):
                    uid, mid, rating, _ = (int(v) for v in ln.strip().split("::"))
                    g, a, j = users[uid]
                    gids, tids = movies[mid]
                    self.data.append(([uid], [g], [a], [j], [mid], gids, tids, [rating * 2 - 5.0]))

    def __getitem__(self, idx):
        return tuple(np.array(d) for d in self.data[idx])

    def __len__(self):
        return len(self.data)


class _LineCorpus(Dataset):
    """Parallel / labelled line corpora stored as tab-separated text inside an archive."""

    def __init__(self, data_file, name, member_pattern):
        _need(data_file, name)
        self.data = []
        opener = zipfile.ZipFile if data_file.endswith(".zip") else tarfile.open
        with opener(data_file) as a:
            members = a.namelist() if isinstance(a, zipfile.ZipFile) else [m.name for m in a.getmembers()]
            for m in members:
                if re.search(member_pattern, m):
                    raw = a.read(m) if isinstance(a, zipfile.ZipFile) else a.extractfile(m).read()
                    for ln in raw.decode("utf-8", "ignore").splitlines():
                        if ln.strip():
                            self.data.append(ln.split("\t"))

    def __getitem__(self, idx):
        return tuple(self.data[idx])

    def __len__(self):
        return len(self.data)


class Conll05st(_LineCorpus):
    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None, target_dict_file=None,
                 emb_file=None, download=True):
        super().__init__(data_file, "Conll05st", r"test\.wsj.*words|props")


class WMT14(_LineCorpus):
    def __init__(self, data_file=None, mode="train", dict_size=-1, download=True):
        super().__init__(data_file, "WMT14", rf"{mode}/{mode}")


class WMT16(_LineCorpus):
    def __init__(self, data_file=None, mode="train", src_dict_size=-1, trg_dict_size=-1, lang="en", download=True):
        super().__init__(data_file, "WMT16", rf"wmt16/{mode}")
