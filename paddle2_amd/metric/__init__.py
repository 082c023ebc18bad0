"""paddle.metric (reference: python/paddle/metric/metrics.py)."""
from __future__ import annotations

import abc

import numpy as np
import torch

from ..framework.tensor import Tensor


def _np(x):
    if isinstance(x, Tensor):
        return x.numpy()
    if isinstance(x, torch.Tensor):
        return x.detach().cpu().numpy()
    return np.asarray(x)


class Metric(abc.ABC):
    def __init__(self):
        pass

    @abc.abstractmethod
    def reset(self):
        ...

    @abc.abstractmethod
    def update(self, *args):
        ...

    @abc.abstractmethod
    def accumulate(self):
        ...

    @abc.abstractmethod
    def name(self):
        ...

    def compute(self, *args):
        return args


class Accuracy(Metric):
    def __init__(self, topk=(1,), name=None, *args, **kwargs):
        super().__init__()
        self.topk = topk
        self.maxk = max(topk)
        self._init_name(name)
        self.reset()

    def compute(self, pred, label, *args):
        p = pred._t if isinstance(pred, Tensor) else torch.as_tensor(pred)
        l = label._t if isinstance(label, Tensor) else torch.as_tensor(label)
        idx = torch.argsort(p, dim=-1, descending=True)[..., : self.maxk]
        if l.dim() == p.dim() and l.shape[-1] == p.shape[-1] and p.shape[-1] > 1:
            l = torch.argmax(l, -1, keepdim=True)
        elif l.dim() == 1 or (l.dim() == p.dim() - 1):
            l = l.reshape(list(l.shape) + [1]) if l.dim() == p.dim() - 1 else l.reshape(-1, 1)
        correct = (idx == l.to(idx.dtype)).float()
        return Tensor._wrap(correct)

    def update(self, correct, *args):
        c = _np(correct)
        num = c.shape[0] if c.ndim > 0 else 1
        accs = []
        for i, k in enumerate(self.topk):
            n = c[..., :k].sum()
            accs.append(float(n) / num)
            self.total[i] += n
            self.count[i] += num
        return accs[0] if len(self.topk) == 1 else accs

    def reset(self):
        self.total = [0.0] * len(self.topk)
        self.count = [0] * len(self.topk)

    def accumulate(self):
        res = [float(t) / c if c > 0 else 0.0 for t, c in zip(self.total, self.count)]
        return res[0] if len(self.topk) == 1 else res

    def _init_name(self, name):
        name = name or "acc"
        self._name = [f"{name}_top{k}" for k in self.topk] if len(self.topk) > 1 else [name]

    def name(self):
        return self._name


class Precision(Metric):
    def __init__(self, name="precision", *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (_np(preds).reshape(-1) > 0.5).astype(np.int64)
        l = _np(labels).reshape(-1).astype(np.int64)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fp += int(((p == 1) & (l == 0)).sum())

    def reset(self):
        self.tp = self.fp = 0

    def accumulate(self):
        ap = self.tp + self.fp
        return float(self.tp) / ap if ap else 0.0

    def name(self):
        return self._name


class Recall(Metric):
    def __init__(self, name="recall", *args, **kwargs):
        super().__init__()
        self._name = name
        self.reset()

    def update(self, preds, labels):
        p = (_np(preds).reshape(-1) > 0.5).astype(np.int64)
        l = _np(labels).reshape(-1).astype(np.int64)
        self.tp += int(((p == 1) & (l == 1)).sum())
        self.fn += int(((p == 0) & (l == 1)).sum())

    def reset(self):
        self.tp = self.fn = 0

    def accumulate(self):
        r = self.tp + self.fn
        return float(self.tp) / r if r else 0.0

    def name(self):
        return self._name


class Auc(Metric):
    def __init__(self, curve="ROC", num_thresholds=4095, name="auc", *args, **kwargs):
        super().__init__()
        self._curve, self._n, self._name = curve, num_thresholds, name
        self.reset()

    def update(self, preds, labels):
        p = _np(preds)
        p = p[:, -1] if p.ndim == 2 else p.reshape(-1)
        l = _np(labels).reshape(-1)
        bins = np.clip((p * self._n).astype(np.int64), 0, self._n)
        for b, y in zip(bins, l):
            if y:
                self._pos[b] += 1
            else:
                self._neg[b] += 1

    def reset(self):
        self._pos = np.zeros(self._n + 1)
        self._neg = np.zeros(self._n + 1)

    def accumulate(self):
        tot_pos = tot_neg = 0.0
        auc = 0.0
        for i in range(self._n, -1, -1):
            np_, nn_ = tot_pos + self._pos[i], tot_neg + self._neg[i]
            auc += (nn_ - tot_neg) * (tot_pos + np_) / 2.0
            tot_pos, tot_neg = np_, nn_
        return auc / (tot_pos * tot_neg) if tot_pos > 0 and tot_neg > 0 else 0.0

    def name(self):
        return self._name


def accuracy(input, label, k=1, correct=None, total=None, name=None):
    p = input._t
    l = label._t.reshape(-1, 1)
    idx = torch.topk(p, k, dim=-1).indices
    c = (idx == l).any(-1).float().mean()
    return Tensor._wrap(c)
