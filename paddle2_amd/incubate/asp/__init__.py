"""paddle.incubate.asp — automatic n:m structured sparsity (reference: python/paddle/incubate/asp/asp.py
``prune_model`` / ``decorate`` / ``set_excluded_layers``, utils.py mask algorithms, supported_layer_list.py).

``prune_model`` computes an n:m mask for every supported weight (Linear, Conv2D and layers registered with
``add_supported_layer``), multiplies it in, and with ``with_mask`` keeps it so that ``decorate(optimizer)``'s step
re-applies it after every update (the pruned weights stay zero through training).  "n:m" means at least n zeros in
every block of m consecutive weights along the REDUCTION dimension of the layer's GEMM (K: a Linear weight's
input dim, a convolution's input channels) — the layout the sparse-matrix instructions consume (gfx950's
``v_smfmac`` 2:4 operand).  Masks:

* ``mask_1d`` — per 1 x m block keep the m - n largest magnitudes;
* ``mask_2d_greedy`` — per m x m block, largest magnitudes first while every row and column of the block keeps at
  most m - n entries;
* ``mask_2d_best`` — per m x m block the valid pattern (every row and column exactly m - n ones) with the largest
  kept magnitude, searched over all such patterns.

Masks are computed with device tensor ops (top-k over blocks), not per-element Python loops; the numpy helpers
(``get_mask_1d``, ``check_mask_1d``, ``create_mask``, ``check_sparsity``, ``calculate_density``) keep the
reference signatures for arrays.
"""
from __future__ import annotations

import itertools
from enum import Enum

import numpy as np
import torch

from ...framework.tensor import Tensor

__all__ = ["calculate_density", "decorate", "prune_model", "set_excluded_layers", "reset_excluded_layers",
           "add_supported_layer", "MaskAlgo", "CheckMethod", "check_mask_1d", "check_mask_2d", "get_mask_1d",
           "get_mask_2d_greedy", "get_mask_2d_best", "create_mask", "check_sparsity", "ASPHelper"]


class MaskAlgo(Enum):
    MASK_1D = "get_mask_1d"
    MASK_2D_GREEDY = "get_mask_2d_greedy"
    MASK_2D_BEST = "get_mask_2d_best"


class CheckMethod(Enum):
    CHECK_1D = "check_mask_1d"
    CHECK_2D = "check_mask_2d"

    @staticmethod
    def get_checking_method(mask_algo):
        return CheckMethod.CHECK_1D if mask_algo == MaskAlgo.MASK_1D else CheckMethod.CHECK_2D


def calculate_density(x):
    x = np.asarray(x._t.detach().cpu() if isinstance(x, Tensor) else x)
    return float(np.count_nonzero(x)) / max(x.size, 1)


# ------------------------------------------------------------------------------------------ masks (torch)
def _pad_cols(t, m):
    r = t.shape[1] % m
    return torch.nn.functional.pad(t, (0, m - r)) if r else t


def _mask_1d_t(t, n, m):
    rows, cols = t.shape
    p = _pad_cols(t.abs(), m)
    blocks = p.reshape(-1, m)
    keep = torch.topk(blocks, m - n, dim=1).indices
    mask = torch.zeros_like(blocks).scatter_(1, keep, 1.0)
    return mask.reshape(rows, -1)[:, :cols]


def _blocks_2d(t, m):
    rows, cols = t.shape
    pr, pc = (-rows) % m, (-cols) % m
    p = torch.nn.functional.pad(t, (0, pc, 0, pr))
    R, C = p.shape
    return p.reshape(R // m, m, C // m, m).permute(0, 2, 1, 3).reshape(-1, m, m), (R, C)


def _unblocks_2d(b, shape, m, out_shape):
    R, C = shape
    return b.reshape(R // m, C // m, m, m).permute(0, 2, 1, 3).reshape(R, C)[:out_shape[0], :out_shape[1]]


def _mask_2d_greedy_t(t, n, m):
    blocks, shape = _blocks_2d(t.abs(), m)
    k = m - n
    nb = blocks.shape[0]
    flat = blocks.reshape(nb, -1)
    order = torch.argsort(flat, dim=1, descending=True)
    mask = torch.zeros_like(flat)
    rc = torch.zeros(nb, m, dtype=torch.int64, device=t.device)
    cc = torch.zeros(nb, m, dtype=torch.int64, device=t.device)
    ar = torch.arange(nb, device=t.device)
    for j in range(m * m):   # m*m vectorised passes over all blocks at once
        e = order[:, j]
        r, c = e // m, e % m
        ok = (rc[ar, r] < k) & (cc[ar, c] < k)
        mask[ar[ok], e[ok]] = 1.0
        rc[ar[ok], r[ok]] += 1
        cc[ar[ok], c[ok]] += 1
    return _unblocks_2d(mask.reshape(nb, m, m), shape, m, t.shape)


_PATTERNS = {}


def _patterns(n, m):
    key = (n, m)
    if key not in _PATTERNS:
        k = m - n
        rows = [r for r in itertools.product([0, 1], repeat=m) if sum(r) == k]
        pats = [p for p in itertools.product(rows, repeat=m) if all(sum(col) == k for col in zip(*p))]
        _PATTERNS[key] = torch.tensor(pats, dtype=torch.float32)   # [P, m, m]
    return _PATTERNS[key]


def _mask_2d_best_t(t, n, m):
    blocks, shape = _blocks_2d(t.abs().float(), m)
    pats = _patterns(n, m).to(t.device)
    score = torch.einsum("bij,pij->bp", blocks, pats)
    best = pats[score.argmax(1)]
    return _unblocks_2d(best, shape, m, t.shape)


_ALGOS = {MaskAlgo.MASK_1D: _mask_1d_t, MaskAlgo.MASK_2D_GREEDY: _mask_2d_greedy_t,
          MaskAlgo.MASK_2D_BEST: _mask_2d_best_t}


def _as2d(t):
    """Reference create_mask layouts: 1-D -> [1, n]; 3-D -> [a*b, c]; 4-D conv (h, w, in, out)-style -> rows over
    the other dims, columns over dim 2 — returns (2-D view, inverse)."""
    shape = t.shape
    if t.dim() == 1:
        return t.reshape(1, -1), lambda x: x.reshape(shape)
    if t.dim() == 2:
        return t, lambda x: x
    if t.dim() == 3:
        return t.reshape(shape[0] * shape[1], shape[2]), lambda x: x.reshape(shape)
    if t.dim() == 4:
        v = t.permute(0, 1, 3, 2).reshape(shape[0] * shape[1] * shape[3], shape[2])
        return v, lambda x: x.reshape(shape[0], shape[1], shape[3], shape[2]).permute(0, 1, 3, 2)
    raise ValueError("create_mask supports tensors of rank <= 4")


def _create_mask_t(t, algo=MaskAlgo.MASK_1D, n=2, m=4):
    v, back = _as2d(t.float())
    return back(_ALGOS[algo](v, n, m)).to(t.dtype)


# ------------------------------------------------------------------------------------------ numpy API
def get_mask_1d(mat, n, m):
    return _mask_1d_t(torch.as_tensor(np.asarray(mat), dtype=torch.float64), n, m).numpy().astype(np.asarray(mat).dtype)


def get_mask_2d_greedy(mat, n, m):
    return _mask_2d_greedy_t(torch.as_tensor(np.asarray(mat), dtype=torch.float64), n, m).numpy().astype(
        np.asarray(mat).dtype)


def get_mask_2d_best(mat, n, m):
    return _mask_2d_best_t(torch.as_tensor(np.asarray(mat), dtype=torch.float64), n, m).numpy().astype(
        np.asarray(mat).dtype)


def check_mask_1d(mat, n, m):
    t = torch.as_tensor(np.asarray(mat)).reshape(1, -1) if np.asarray(mat).ndim <= 1 else torch.as_tensor(
        np.asarray(mat))
    blocks = _pad_cols((t != 0).float(), m).reshape(-1, m)
    return bool((blocks.sum(1) <= m - n).all())


def check_mask_2d(mat, n, m):
    t = torch.as_tensor(np.asarray(mat))
    blocks, _ = _blocks_2d((t != 0).float(), m)
    return bool((blocks.sum(1) <= m - n).all() and (blocks.sum(2) <= m - n).all())


def create_mask(tensor, func_name=MaskAlgo.MASK_1D, n=2, m=4):
    if not isinstance(func_name, MaskAlgo):
        raise TypeError(f"func_name must be a MaskAlgo, got {type(func_name)}")
    arr = np.asarray(tensor)
    return _create_mask_t(torch.as_tensor(arr, dtype=torch.float64), func_name, n, m).numpy().astype(arr.dtype)


def check_sparsity(tensor, func_name=CheckMethod.CHECK_1D, n=2, m=4):
    if not isinstance(func_name, CheckMethod):
        raise TypeError(f"func_name must be a CheckMethod, got {type(func_name)}")
    v, _ = _as2d(torch.as_tensor(np.asarray(tensor)))
    fn = check_mask_1d if func_name == CheckMethod.CHECK_1D else check_mask_2d
    return fn(v.numpy(), n, m)


# ------------------------------------------------------------------------------------------ layers / helper
def _linear_pruner(weight, n, m, algo):
    """Linear weight [in, out]: n:m along `in` (K) for every output column."""
    return _create_mask_t(weight.t(), algo, n, m).t()


def _conv_pruner(weight, n, m, algo):
    """Conv weight [out, in, kh, kw]: n:m along the input channels for every (out, kh, kw)."""
    o, i, kh, kw = weight.shape
    v = weight.permute(0, 2, 3, 1).reshape(-1, i)
    mask = _create_mask_t(v, algo, n, m)
    return mask.reshape(o, kh, kw, i).permute(0, 3, 1, 2)


class ASPHelper:
    """Registry of supported layers, excluded parameters and the masks of pruned parameters (reference
    asp.py:536)."""

    _supported = {}        # layer class name -> pruning fn (weight, n, m, algo) -> mask
    _excluded = set()      # parameter names
    _masks = {}            # parameter name -> (parameter, mask tensor)

    @classmethod
    def _pruner_of(cls, layer):
        for klass in type(layer).__mro__:
            fn = cls._supported.get(klass.__name__)
            if fn is not None:
                return fn
        return None

    @classmethod
    def _is_supported(cls, layer):
        return cls._pruner_of(layer) is not None


def add_supported_layer(layer, pruning_func=None):
    """Register a layer class (or its name) for pruning; ``pruning_func(weight, n, m, mask_algo) -> mask`` (a
    torch tensor of the weight's shape) overrides the default 1-D pruning along the weight's last dim."""
    name = layer if isinstance(layer, str) else (layer.__name__ if isinstance(layer, type) else type(layer).__name__)

    def default(w, n, m, algo):
        return _create_mask_t(w, algo, n, m)

    if pruning_func is None:
        ASPHelper._supported[name] = default
    else:
        def wrapped(w, n, m, algo):
            out = pruning_func(Tensor._wrap(w), n, m, algo.value if isinstance(algo, MaskAlgo) else algo, "")
            if isinstance(out, tuple):
                out = out[1]
            return torch.as_tensor(np.asarray(out._t.cpu() if isinstance(out, Tensor) else out),
                                   dtype=w.dtype, device=w.device)

        ASPHelper._supported[name] = wrapped


ASPHelper._supported.update({"Linear": _linear_pruner, "Conv2D": _conv_pruner})


def set_excluded_layers(param_names=None, main_program=None):
    """Parameters (by name, or every parameter of the given layers) that prune_model must skip."""
    names = param_names if isinstance(param_names, (list, tuple)) else [param_names]
    for n in names:
        if n is None:
            continue
        if hasattr(n, "parameters"):
            ASPHelper._excluded.update(p.name for p in n.parameters())
        else:
            ASPHelper._excluded.add(n)


def reset_excluded_layers(main_program=None):
    ASPHelper._excluded.clear()


@torch.no_grad()
def prune_model(model, n=2, m=4, mask_algo="mask_1d", with_mask=True):
    """Prune every supported layer's weight of ``model`` to the n:m pattern; -> {param name: mask Tensor}."""
    algo = {"mask_1d": MaskAlgo.MASK_1D, "mask_2d_greedy": MaskAlgo.MASK_2D_GREEDY,
            "mask_2d_best": MaskAlgo.MASK_2D_BEST}.get(mask_algo, mask_algo)
    if not isinstance(algo, MaskAlgo):
        raise ValueError(f"unknown mask_algo {mask_algo!r}")
    out = {}
    layers = model.sublayers(include_self=True) if hasattr(model, "sublayers") else []
    for layer in layers:
        fn = ASPHelper._pruner_of(layer)
        w = getattr(layer, "weight", None)
        if fn is None or w is None or w.name in ASPHelper._excluded:
            continue
        if w._t.dim() < 2:
            continue
        mask = fn(w._t, n, m, algo).to(w._t.dtype)
        w._t.mul_(mask)
        out[w.name] = Tensor._wrap(mask)
        if with_mask:
            ASPHelper._masks[w.name] = (w, mask)
    return out


class OptimizerWithSparsityGuarantee:
    """``decorate(optimizer)``: every step re-applies the pruning masks to the updated weights."""

    def __init__(self, optimizer):
        self._optimizer = optimizer

    def __getattr__(self, name):
        return getattr(self._optimizer, name)

    @torch.no_grad()
    def _apply_masks(self):
        for w, mask in ASPHelper._masks.values():
            w._t.mul_(mask)

    def step(self):
        self._optimizer.step()
        self._apply_masks()

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        out = self._optimizer.minimize(loss, startup_program, parameters, no_grad_set)
        self._apply_masks()
        return out

    def clear_grad(self, set_to_zero=True):
        self._optimizer.clear_grad(set_to_zero)

    def state_dict(self):
        sd = self._optimizer.state_dict()
        for name, (_, mask) in ASPHelper._masks.items():
            sd[f"{name}_asp_mask"] = Tensor._wrap(mask)
        return sd


def decorate(optimizer):
    return OptimizerWithSparsityGuarantee(optimizer)
