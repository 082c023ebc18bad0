"""paddle.dataset.movielens: readers over paddle.text.datasets.Movielens (reference dataset/movielens.py); the archive is read
from common.DATA_HOME/movielens/ml-1m.zip."""
from . import common

__all__ = ["train", "test"]


def _reader(mode, **kw):
    def r():
        from ..text.datasets import Movielens

        ds = Movielens(data_file=common._local("movielens", "ml-1m.zip"), mode=mode, **kw)
        for i in range(len(ds)):
            yield tuple(ds[i])

    return r


def train(**kw):
    return _reader("train", **kw)


def test(**kw):
    return _reader("test", **kw)
