"""BaseObserver (reference: python/paddle/quantization/base_observer.py): a quanter that only records statistics
during calibration (PTQ) and turns them into thresholds."""
from __future__ import annotations

import abc

from .base_quanter import BaseQuanter


class BaseObserver(BaseQuanter, metaclass=abc.ABCMeta):
    def __init__(self):
        super().__init__()

    @abc.abstractmethod
    def cal_thresholds(self):
        ...
