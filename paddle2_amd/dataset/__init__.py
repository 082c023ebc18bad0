"""paddle.dataset — the legacy reader-creator datasets (reference: python/paddle/dataset/{common,mnist,cifar,
uci_housing,imdb,imikolov,movielens,conll05,wmt14,wmt16}.py): ``train()`` / ``test()`` return readers (callables
yielding samples) over the same parsers as ``paddle.vision.datasets`` / ``paddle.text.datasets``.  Files are read
from ``common.DATA_HOME/<module>/`` (nothing is downloaded here)."""
from . import cifar, common, conll05, imdb, imikolov, mnist, movielens, uci_housing, wmt14, wmt16  # noqa: F401

__all__ = ["common", "mnist", "cifar", "uci_housing", "imdb", "imikolov", "movielens", "conll05", "wmt14", "wmt16"]
