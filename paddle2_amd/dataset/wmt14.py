"""paddle.dataset.wmt14: readers over paddle.text.datasets.WMT14 (reference dataset/wmt14.py)."""
from . import common

__all__ = ["train", "test", "gen"]


def _reader(mode, dict_size):
    def r():
        from ..text.datasets import WMT14

        ds = WMT14(common._local("wmt14", "wmt14.tgz"), mode, dict_size)
        for i in range(len(ds)):
            yield tuple(x.tolist() for x in ds[i])

    return r


def train(dict_size):
    return _reader("train", dict_size)


def test(dict_size):
    return _reader("test", dict_size)


def gen(dict_size):
    return _reader("gen", dict_size)
