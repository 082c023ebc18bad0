"""paddle.dataset.wmt16: readers over paddle.text.datasets.WMT16 (reference dataset/wmt16.py)."""
from . import common

__all__ = ["train", "test", "validation"]


def _reader(mode, src_dict_size, trg_dict_size, src_lang):
    def r():
        from ..text.datasets import WMT16

        ds = WMT16(common._local("wmt16", "wmt16.tar.gz"), mode, src_dict_size, trg_dict_size, src_lang)
        for i in range(len(ds)):
            yield tuple(x.tolist() for x in ds[i])

    return r


def train(src_dict_size, trg_dict_size, src_lang="en"):
    return _reader("train", src_dict_size, trg_dict_size, src_lang)


def test(src_dict_size, trg_dict_size, src_lang="en"):
    return _reader("test", src_dict_size, trg_dict_size, src_lang)


def validation(src_dict_size, trg_dict_size, src_lang="en"):
    return _reader("val", src_dict_size, trg_dict_size, src_lang)
