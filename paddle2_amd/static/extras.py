"""Remaining paddle.static API (reference python/paddle/static/__init__.py __all__): Print, WeightNormParamAttr,
ExponentialMovingAverage, save_to_file / load_from_file, normalize_program, accuracy / auc / ctr_metric_bundle,
xpu_places and the IPU entry points (no IPU on this target: they raise)."""
from __future__ import annotations

import torch

from ..framework.param import ParamAttr
from ..framework.tensor import Tensor


def Print(input, first_n=-1, message=None, summarize=20, print_tensor_name=True, print_tensor_type=True,  # noqa: A002,N802
          print_tensor_shape=True, print_tensor_lod=True, print_phase="both"):
    from ..ops.extra_ops import print_op as _p

    return _p(input, first_n, message or "", summarize, print_tensor_name, print_tensor_type, print_tensor_shape)


class WeightNormParamAttr(ParamAttr):
    """ParamAttr for weight-normalised parameters: ``dim`` is the axis the norm is kept along
    (nn.utils.weight_norm applies it in dygraph)."""

    def __init__(self, dim=None, name=None, initializer=None, learning_rate=1.0, regularizer=None, trainable=True,
                 do_model_average=False, need_clip=True):
        super().__init__(name=name, initializer=initializer, learning_rate=learning_rate, regularizer=regularizer,
                         trainable=trainable, need_clip=need_clip)
        self.dim = dim
        self.do_model_average = do_model_average


class ExponentialMovingAverage:
    """Shadow weights ema = decay * ema + (1 - decay) * param (with the reference's thres_steps bias-free decay
    min(decay, (1 + step) / (10 + step))); ``apply()`` swaps the averages in (a context manager restoring the
    trained weights on exit unless need_restore=False), ``restore()`` swaps back."""

    def __init__(self, decay=0.999, thres_steps=None, name=None, parameters=None):
        self._decay = decay
        self._thres = thres_steps
        self._params = list(parameters) if parameters is not None else None
        self._ema = {}
        self._backup = {}
        self._step = 0

    def _plist(self):
        if self._params is None:
            raise ValueError("ExponentialMovingAverage needs parameters= in this framework")
        return self._params

    @torch.no_grad()
    def update(self):
        self._step += 1
        d = self._decay
        if self._thres is not None:
            d = min(d, (1.0 + self._step) / (10.0 + self._step))
        for p in self._plist():
            t = p._t.detach().float()
            e = self._ema.get(id(p))
            self._ema[id(p)] = t.clone() if e is None else e.mul_(d).add_(t, alpha=1 - d)

    def apply(self, executor=None, need_restore=True):
        ema = self

        class _Ctx:
            def __enter__(self_):
                with torch.no_grad():
                    for p in ema._plist():
                        if id(p) in ema._ema:
                            ema._backup[id(p)] = p._t.detach().clone()
                            p._t.copy_(ema._ema[id(p)].to(p._t.dtype))
                return self_

            def __exit__(self_, *a):
                if need_restore:
                    ema.restore()
                return False

        return _Ctx()

    @torch.no_grad()
    def restore(self, executor=None):
        for p in self._plist():
            b = self._backup.pop(id(p), None)
            if b is not None:
                p._t.copy_(b)


def save_to_file(path, content):
    with open(path, "wb") as f:
        f.write(content if isinstance(content, (bytes, bytearray)) else bytes(content))


def load_from_file(path):
    with open(path, "rb") as f:
        return f.read()


def normalize_program(program, feed_vars, fetch_vars, **kwargs):
    """Inference form of a Program: training-only ops dropped (clone(for_test=True)) and the feed / fetch
    interface recorded on it."""
    p = program.clone(for_test=True)
    p._feed_names = [getattr(v, "name", None) or v for v in (feed_vars or [])]
    p._fetch_vars = list(fetch_vars or [])
    return p


def xpu_places(device_ids=None):
    return []


def accuracy(input, label, k=1, correct=None, total=None):  # noqa: A002
    from ..metric import accuracy as _acc

    return _acc(input, label, k, correct, total)


def auc(input, label, curve="ROC", num_thresholds=2 ** 12 - 1, topk=1, slide_steps=1, ins_tag_weight=None):  # noqa: A002
    """Returns (auc, batch_auc, [stat_pos, stat_neg, ...]) like the reference static.auc (batch_auc over this
    batch alone; the streaming statistics start empty per call here)."""
    from ..ops.extra_ops import auc as _auc

    sp = torch.zeros(num_thresholds + 1, dtype=torch.int64)
    sn = torch.zeros(num_thresholds + 1, dtype=torch.int64)
    a, sp_, sn_ = _auc(input, label, Tensor._wrap(sp), Tensor._wrap(sn), curve=curve, num_thresholds=num_thresholds)
    return a, a, [sp_, sn_]


def ctr_metric_bundle(input, label, ins_tag_weight=None):  # noqa: A002
    """CTR metrics of a batch: (sqrerr, abserr, prob sum, q sum, positive count, instance count)."""
    p = (input._t if isinstance(input, Tensor) else input).float().reshape(-1)
    y = (label._t if isinstance(label, Tensor) else label).float().reshape(-1)
    w = lambda v: Tensor._wrap(torch.as_tensor([float(v)]))  # noqa: E731
    q = torch.log(p.clamp_min(1e-12) / (1 - p).clamp_min(1e-12))
    return (w(((p - y) ** 2).sum()), w((p - y).abs().sum()), w(p.sum()), w(q.sum()), w(y.sum()), w(y.numel()))


class IpuStrategy:
    def __init__(self, *a, **k):
        raise RuntimeError("IpuStrategy: Graphcore IPUs are not a target of this framework (MI355X only)")


class IpuCompiledProgram:
    def __init__(self, *a, **k):
        raise RuntimeError("IpuCompiledProgram: Graphcore IPUs are not a target of this framework (MI355X only)")


def set_ipu_shard(call_func, index=-1, stage=-1):
    raise RuntimeError("set_ipu_shard: Graphcore IPUs are not a target of this framework (MI355X only)")
