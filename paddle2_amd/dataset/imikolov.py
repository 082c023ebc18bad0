"""paddle.dataset.imikolov: readers over paddle.text.datasets.Imikolov (reference dataset/imikolov.py); the archive is read
from common.DATA_HOME/imikolov/simple-examples.tgz."""
from . import common

__all__ = ["train", "test"]


def _reader(mode, **kw):
    def r():
        from ..text.datasets import Imikolov

        ds = Imikolov(data_file=common._local("imikolov", "simple-examples.tgz"), mode=mode, **kw)
        for i in range(len(ds)):
            yield tuple(ds[i])

    return r


def train(**kw):
    return _reader("train", **kw)


def test(**kw):
    return _reader("test", **kw)
