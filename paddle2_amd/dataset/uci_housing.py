"""paddle.dataset.uci_housing: readers over paddle.text.datasets.UCIHousing (reference dataset/uci_housing.py); the archive is read
from common.DATA_HOME/uci_housing/housing.data."""
from . import common

__all__ = ["train", "test"]


def _reader(mode, **kw):
    def r():
        from ..text.datasets import UCIHousing

        ds = UCIHousing(data_file=common._local("uci_housing", "housing.data"), mode=mode, **kw)
        for i in range(len(ds)):
            yield tuple(ds[i])

    return r


def train(**kw):
    return _reader("train", **kw)


def test(**kw):
    return _reader("test", **kw)
