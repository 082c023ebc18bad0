"""Text datasets (reference: python/paddle/text/datasets/{uci_housing,imdb,imikolov,movielens,
conll05,wmt14,wmt16}.py).

There is no network here: every dataset reads a local copy of the official archive via
``data_file=`` (the reference's download cache path) and raises a clear error when it is missing.
Every dataset parses its official archive layout (dictionaries, tab-separated pairs, gzipped CoNLL columns).
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


_S, _E, _U = "<s>", "<e>", "<unk>"


def _tar_lines(tf, name):
    for ln in tf.extractfile(name):
        yield ln.decode("utf-8", "ignore")


def _pairs_to_ids(lines, src_dict, trg_dict, src_col, unk, max_len=None):
    """Tab-separated sentence pairs -> (src, trg, trg_next) id lists with <s>/<e> framing."""
    src_ids, trg_ids, trg_next = [], [], []
    s_id, e_id = src_dict[_S], src_dict[_E]
    for ln in lines:
        cols = ln.strip().split("\t")
        if len(cols) != 2:
            continue
        src = [s_id] + [src_dict.get(w, unk) for w in cols[src_col].split()] + [e_id]
        trg = [trg_dict.get(w, unk) for w in cols[1 - src_col].split()]
        if max_len is not None and (len(src) > max_len or len(trg) > max_len):
            continue
        src_ids.append(src)
        trg_ids.append([trg_dict.get(_S, s_id)] + trg)
        trg_next.append(trg + [trg_dict.get(_E, e_id)])
    return src_ids, trg_ids, trg_next


class _Seq2Seq(Dataset):
    def __getitem__(self, idx):
        return np.array(self.src_ids[idx]), np.array(self.trg_ids[idx]), np.array(self.trg_ids_next[idx])

    def __len__(self):
        return len(self.src_ids)


class WMT14(_Seq2Seq):
    """WMT14 en-fr (reference text/datasets/wmt14.py:113-215): the archive's ``src.dict`` / ``trg.dict`` give the
    first ``dict_size`` words their line numbers; ``{mode}/{mode}`` holds tab-separated pairs; pairs longer than 80
    ids are dropped.  Items: (src ids with <s>..<e>, <s> + trg ids, trg ids + <e>)."""

    def __init__(self, data_file=None, mode="train", dict_size=-1, download=True):
        mode = mode.lower()
        if mode not in ("train", "test", "gen"):
            raise ValueError(f"mode should be 'train', 'test' or 'gen', but got {mode}")
        _need(data_file, "WMT14")
        if dict_size <= 0:
            raise ValueError("dict_size should be set as positive number")
        self.mode, self.data_file, self.dict_size = mode, data_file, dict_size
        with tarfile.open(data_file) as tf:
            names = [m.name for m in tf.getmembers()]

            def read_dict(suffix):
                (name,) = [n for n in names if n.endswith(suffix)]
                out = {}
                for i, ln in enumerate(_tar_lines(tf, name)):
                    if i >= dict_size:
                        break
                    out[ln.strip()] = i
                return out

            self.src_dict, self.trg_dict = read_dict("src.dict"), read_dict("trg.dict")
            self.src_ids, self.trg_ids, self.trg_ids_next = [], [], []
            for name in (n for n in names if n.endswith(f"{mode}/{mode}")):
                a, b, c = _pairs_to_ids(_tar_lines(tf, name), self.src_dict, self.trg_dict, 0, 2, max_len=80)
                self.src_ids += a
                self.trg_ids += b
                self.trg_ids_next += c

    def get_dict(self, reverse=False):
        if reverse:
            return {v: k for k, v in self.src_dict.items()}, {v: k for k, v in self.trg_dict.items()}
        return self.src_dict, self.trg_dict


class WMT16(_Seq2Seq):
    """WMT16 en-de (reference text/datasets/wmt16.py:130-339): word dictionaries are built from ``wmt16/train``
    by descending frequency after the three marks (<s>, <e>, <unk>), ``dict_size`` entries in total; ``lang``
    picks the source column.  Dictionaries are kept in memory (and cached per archive / size in this process)."""

    TOTAL_EN_WORDS, TOTAL_DE_WORDS = 11250, 19220
    _dict_cache = {}

    def __init__(self, data_file=None, mode="train", src_dict_size=-1, trg_dict_size=-1, lang="en", download=True):
        mode = mode.lower()
        if mode not in ("train", "test", "val"):
            raise ValueError(f"mode should be 'train', 'test' or 'val', but got {mode}")
        if lang not in ("en", "de"):
            raise ValueError(f"lang should be 'en' or 'de', but got {lang}")
        _need(data_file, "WMT16")
        if src_dict_size <= 0 or trg_dict_size <= 0:
            raise ValueError("dict_size should be set as positive number")
        self.mode, self.data_file, self.lang = mode, data_file, lang
        other = "de" if lang == "en" else "en"
        total = {"en": self.TOTAL_EN_WORDS, "de": self.TOTAL_DE_WORDS}
        self.src_dict_size = min(src_dict_size, total[lang])
        self.trg_dict_size = min(trg_dict_size, total[other])
        self.src_dict = self._load_dict(lang, src_dict_size)
        self.trg_dict = self._load_dict(other, trg_dict_size)
        with tarfile.open(data_file) as tf:
            self.src_ids, self.trg_ids, self.trg_ids_next = _pairs_to_ids(
                _tar_lines(tf, f"wmt16/{mode}"), self.src_dict, self.trg_dict, 0 if lang == "en" else 1,
                self.src_dict[_U])

    def _load_dict(self, lang, dict_size, reverse=False):
        key = (os.path.abspath(self.data_file), lang, dict_size)
        d = self._dict_cache.get(key)
        if d is None:
            counts = collections.Counter()
            col = 0 if lang == "en" else 1
            with tarfile.open(self.data_file) as tf:
                for ln in _tar_lines(tf, "wmt16/train"):
                    cols = ln.strip().split("\t")
                    if len(cols) == 2:
                        counts.update(cols[col].split())
            words = [_S, _E, _U] + [w for w, _ in sorted(counts.items(), key=lambda x: -x[1])][:max(dict_size - 3, 0)]
            d = self._dict_cache[key] = {w: i for i, w in enumerate(words)}
        return {i: w for w, i in d.items()} if reverse else dict(d)

    def get_dict(self, lang, reverse=False):
        size = self.src_dict_size if lang == self.lang else self.trg_dict_size
        return self._load_dict(lang, size, reverse)


class Conll05st(Dataset):
    """CoNLL-2005 semantic role labelling, WSJ test split (reference text/datasets/conll05.py:125-397).

    ``test.wsj.words.gz`` / ``test.wsj.props.gz`` inside the archive are read in lock-step; a blank props line ends
    a sentence, whose first props column marks the predicates and every further column is one predicate's bracketed
    argument spans, turned into B-/I-/O tags.  Items are the nine id sequences of the reference's SRL model: words,
    the five-word context window around the verb (each repeated over the sentence), the predicate, the window mark,
    and the tag ids.  The label dictionary orders its tags by name (the reference iterates a set, whose order is
    not fixed across interpreter runs)."""

    UNK_IDX = 0

    def __init__(self, data_file=None, word_dict_file=None, verb_dict_file=None, target_dict_file=None,
                 emb_file=None, download=True):
        for f, n in ((data_file, "Conll05st data_file"), (word_dict_file, "Conll05st word_dict_file"),
                     (verb_dict_file, "Conll05st verb_dict_file"), (target_dict_file, "Conll05st target_dict_file")):
            _need(f, n)
        self.data_file, self.emb_file = data_file, emb_file
        self.word_dict_file, self.verb_dict_file, self.target_dict_file = word_dict_file, verb_dict_file, \
            target_dict_file
        self.word_dict = self._load_dict(word_dict_file)
        self.predicate_dict = self._load_dict(verb_dict_file)
        self.label_dict = self._load_label_dict(target_dict_file)
        self._load_anno()

    @staticmethod
    def _load_dict(filename):
        with open(filename) as f:
            return {ln.strip(): i for i, ln in enumerate(f)}

    @staticmethod
    def _load_label_dict(filename):
        tags = set()
        with open(filename) as f:
            for ln in f:
                ln = ln.strip()
                if ln[:2] in ("B-", "I-"):
                    tags.add(ln[2:])
        d = {}
        for t in sorted(tags):
            d["B-" + t] = len(d)
            d["I-" + t] = len(d)
        d["O"] = len(d)
        return d

    @staticmethod
    def _bio(column):
        """One predicate's props column (``(A0*``, ``*``, ``*)``, ``(V*)``) -> B-/I-/O tags."""
        out, tag, open_ = [], "O", False
        for tok in column:
            if tok == "*":
                out.append("I-" + tag if open_ else "O")
            elif tok == "*)":
                out.append("I-" + tag)
                open_ = False
            elif "(" in tok:
                tag = tok[1:tok.index("*")]
                out.append("B-" + tag)
                open_ = ")" not in tok
            else:
                raise RuntimeError(f"Unexpected label: {tok}")
        return out

    def _load_anno(self):
        import gzip

        self.sentences, self.predicates, self.labels = [], [], []
        base = "conll05st-release/test.wsj"
        with tarfile.open(self.data_file) as tf, \
                gzip.GzipFile(fileobj=tf.extractfile(f"{base}/words/test.wsj.words.gz")) as wf, \
                gzip.GzipFile(fileobj=tf.extractfile(f"{base}/props/test.wsj.props.gz")) as pf:
            words, rows = [], []
            for w, p in zip(wf, pf):
                w, cols = w.decode().strip(), p.decode().split()
                if cols:
                    words.append(w)
                    rows.append(cols)
                    continue
                if rows:
                    columns = list(zip(*rows))
                    verbs = [x for x in columns[0] if x != "-"]
                    for k, col in enumerate(columns[1:]):
                        self.sentences.append(words)
                        self.predicates.append(verbs[k])
                        self.labels.append(self._bio(col))
                words, rows = [], []

    def __getitem__(self, idx):
        sent, pred, labels = self.sentences[idx], self.predicates[idx], self.labels[idx]
        n = len(sent)
        v = labels.index("B-V")
        mark = [0] * n
        ctx = []
        for off in (-2, -1, 0, 1, 2):
            j = v + off
            if 0 <= j < n:
                mark[j] = 1
                ctx.append(sent[j])
            else:
                ctx.append("bos" if off < 0 else "eos")
        wd = self.word_dict
        out = [[wd.get(w, self.UNK_IDX) for w in sent]]
        out += [[wd.get(c, self.UNK_IDX)] * n for c in ctx]
        out += [[self.predicate_dict.get(pred)] * n, mark, [self.label_dict.get(t) for t in labels]]
        return tuple(np.array(x) for x in out)

    def __len__(self):
        return len(self.sentences)

    def get_dict(self):
        return self.word_dict, self.predicate_dict, self.label_dict

    def get_embedding(self):
        return self.emb_file
