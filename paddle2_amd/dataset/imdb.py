"""paddle.dataset.imdb: readers over paddle.text.datasets.Imdb (reference dataset/imdb.py); the archive is read
from common.DATA_HOME/imdb/aclImdb_v1.tar.gz."""
from . import common

__all__ = ["train", "test"]


def _reader(mode, **kw):
    def r():
        from ..text.datasets import Imdb

        ds = Imdb(data_file=common._local("imdb", "aclImdb_v1.tar.gz"), mode=mode, **kw)
        for i in range(len(ds)):
            yield tuple(ds[i])

    return r


def train(**kw):
    return _reader("train", **kw)


def test(**kw):
    return _reader("test", **kw)
