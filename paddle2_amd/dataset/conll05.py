"""paddle.dataset.conll05: the test-split reader over paddle.text.datasets.Conll05st (reference
dataset/conll05.py)."""
from . import common

__all__ = ["test", "get_dict", "get_embedding"]


def _ds():
    from ..text.datasets import Conll05st

    return Conll05st(common._local("conll05st", "conll05st-tests.tar.gz"), common._local("conll05st", "wordDict.txt"),
                     common._local("conll05st", "verbDict.txt"), common._local("conll05st", "targetDict.txt"),
                     common._local("conll05st", "emb"))


def test():
    def r():
        ds = _ds()
        for i in range(len(ds)):
            yield tuple(x.tolist() for x in ds[i])

    return r


def get_dict():
    return _ds().get_dict()


def get_embedding():
    return common._local("conll05st", "emb")
