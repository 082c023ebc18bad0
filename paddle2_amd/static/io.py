"""Static Program serialization (reference: python/paddle/static/io.py ``save_inference_model`` /
``load_inference_model`` writing ``{prefix}.pdmodel`` + ``{prefix}.pdiparams``).

``.pdmodel`` here stores the pruned op list with every callable as a NAME (torch op, tensor
method / attribute, or a paddle2_amd native-kernel entry point), variables as ids and tensors as
references into ``.pdiparams`` (a paddle.save state dict), so loading executes no code from the
file: the model file is read with an allowlisting unpickler and names are resolved against
torch / paddle2_amd only.
"""
from __future__ import annotations

import importlib
import io as _io
import pickle

import torch
from torch.utils import _pytree as pytree

from ..framework.tensor import Tensor
from .graph import Op, Program, SymTensor, VarRef

_FORMAT = "paddle2_amd.static.v1"


# ----------------------------------------------------------------------------- callable names
def _fn_name(fn):
    if getattr(fn, "_graph_op", False):
        return f"{fn.__module__}:{fn.__qualname__}"
    qn0 = getattr(fn, "__qualname__", "") or ""
    if getattr(fn, "__module__", "") == "torch" and "." in qn0:
        return f"torch:{fn.__name__}"  # builtins exposed as torch.<name> (_VariableFunctionsClass.<name>)
    if getattr(fn, "__module__", "") in ("torch", "torch.nn.functional"):
        if "<locals>" in qn0:  # e.g. boolean_dispatch wrappers (F.max_pool2d): resolve by public name
            return f"{fn.__module__}:{fn.__name__}"
        return f"{fn.__module__}:{qn0}"
    self_ = getattr(fn, "__self__", None)
    if type(fn).__name__ == "method-wrapper" and self_ is not None and hasattr(self_, "__objclass__"):
        return f"getattr:{self_.__name__}"  # getset_descriptor.__get__ (x.T, x.mT, x.real ...)
    qn = getattr(fn, "__qualname__", "")
    name = getattr(fn, "__name__", "")
    if qn.startswith("TensorBase.") or qn.startswith("Tensor."):
        return f"tensor:{name}"
    if qn.startswith("_VariableFunctionsClass.") or qn.startswith("_VariableFunctions."):
        return f"torch:{name}"
    mod = getattr(fn, "__module__", None)
    if mod and (mod.startswith("torch") or mod.startswith("paddle2_amd")):
        return f"{mod}:{qn}"
    raise ValueError(f"cannot serialize op callable {fn!r}")


def _resolve(name):
    kind, _, rest = name.partition(":")
    if kind == "getattr":
        return lambda t: getattr(t, rest)
    if kind == "tensor":
        return getattr(torch.Tensor, rest)
    if kind == "torch" and "." not in rest:
        return getattr(torch, rest)
    if not (kind.startswith("torch") or kind.startswith("paddle2_amd")):
        raise ValueError(f"refusing to resolve {name}")
    obj = importlib.import_module(kind)
    for part in rest.split("."):
        obj = getattr(obj, part)
    return obj


# ----------------------------------------------------------------------------- pruning
def _prune(program, fetch_ids):
    need = set(fetch_ids)
    keep = []
    for op in reversed(program.ops):
        if op.kind not in ("torch", "native"):
            continue
        if op.attrs.get("side_effect") or any(o in need for o in op.outs if o is not None):
            keep.append(op)
            for x in pytree.tree_leaves((op.args, op.kwargs)):
                if isinstance(x, VarRef):
                    need.add(x.vid)
    return list(reversed(keep))


class _TensorRef:
    __slots__ = ("name",)

    def __init__(self, name):
        self.name = name


def serialize_program(feed_vars, fetch_vars, program=None, **kw):
    from .graph import default_main_program

    program = program or default_main_program()
    fetch_ids = [f._t._vid for f in fetch_vars]
    ops = _prune(program, fetch_ids)
    tensors, names = {}, {}

    def enc(x):
        if isinstance(x, torch.Tensor) and not isinstance(x, SymTensor):
            key = id(x)
            if key not in names:
                p = getattr(x, "_pd_param", None)
                nm = p.name if p is not None else f"__const_{len(names)}"
                names[key] = nm
                tensors[nm] = x.detach()
            return _TensorRef(names[key])
        if isinstance(x, torch.dtype):
            return ("__dtype__", str(x).replace("torch.", ""))
        if isinstance(x, torch.device):
            return ("__device__", x.type)
        return x

    rec = []
    for op in ops:
        rec.append((op.kind, _fn_name(op.fn), pytree.tree_map(enc, op.args), pytree.tree_map(enc, op.kwargs),
                    list(op.outs)))
    feeds = {}
    for v in feed_vars:
        s = v._t
        feeds[s._name] = (s._vid, list(s.shape), str(s.dtype).replace("torch.", ""))
    model = {"format": _FORMAT, "ops": rec, "feeds": feeds, "fetch": fetch_ids}
    buf = _io.BytesIO()
    pickle.dump(model, buf, protocol=4)
    return buf.getvalue(), tensors


def serialize_persistables(feed_vars, fetch_vars, executor=None, program=None, **kw):
    _, tensors = serialize_program(feed_vars, fetch_vars, program)
    buf = _io.BytesIO()
    from ..framework.io import save as _save

    _save({k: Tensor._wrap(v) for k, v in tensors.items()}, buf)
    return buf.getvalue()


def save_inference_model(path_prefix, feed_vars, fetch_vars, executor=None, program=None, **kwargs):
    """Writes the reference format (ProgramDesc ``.pdmodel`` + save_combine ``.pdiparams``, static/pdmodel.py) when
    every op lowers to a Paddle op type; otherwise (``format="native"`` or an op outside the lowering table) the
    framework's own op-list program."""
    from ..framework.io import save as _save
    from . import pdmodel
    from .graph import default_main_program

    feed_vars = feed_vars if isinstance(feed_vars, (list, tuple)) else [feed_vars]
    fetch_vars = fetch_vars if isinstance(fetch_vars, (list, tuple)) else [fetch_vars]
    if kwargs.get("format", "paddle") == "paddle":
        prog = program or default_main_program()
        fetch_ids = [f._t._vid for f in fetch_vars]
        feeds = {v._t._name: v._t for v in feed_vars}
        try:
            pdmodel.save(path_prefix, prog, _prune(prog, fetch_ids), feeds, fetch_ids, _fn_name)
            return
        except pdmodel.Unmapped as e:
            import warnings

            warnings.warn(f"save_inference_model: {e} has no Paddle op mapping; writing the native program format")
    model, tensors = serialize_program(feed_vars, fetch_vars, program)
    with open(path_prefix + ".pdmodel", "wb") as f:
        f.write(model)
    _save({k: Tensor._wrap(v.cpu()) for k, v in tensors.items()}, path_prefix + ".pdiparams")


class _ModelUnpickler(pickle.Unpickler):
    _OK = {("builtins", "list"), ("builtins", "dict"), ("builtins", "tuple"), ("builtins", "slice"),
           ("builtins", "Ellipsis"), ("builtins", "set")}

    def find_class(self, module, name):
        if module == __name__ and name in ("_TensorRef",):
            return _TensorRef
        if module == "paddle2_amd.static.graph" and name == "VarRef":
            return VarRef
        if (module, name) in self._OK:
            import builtins

            return getattr(builtins, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a model file")


def deserialize_program(data, tensors=None, device=None):
    model = _ModelUnpickler(_io.BytesIO(data)).load()
    assert model.get("format") == _FORMAT, "unknown model format"
    tensors = tensors or {}
    from ..framework.dtype import convert_dtype

    def dec(x):
        if isinstance(x, _TensorRef):
            t = tensors[x.name]
            return t._t if isinstance(t, Tensor) else t
        if isinstance(x, tuple) and len(x) == 2 and x[0] == "__dtype__":
            return convert_dtype(x[1])
        if isinstance(x, tuple) and len(x) == 2 and x[0] == "__device__":
            return device if device is not None else torch.device(x[1])
        return x

    prog = Program()
    for kind, fname, args, kwargs, outs in model["ops"]:
        prog.ops.append(Op(kind, _resolve(fname), pytree.tree_map(dec, args, is_leaf=lambda z: isinstance(
            z, (_TensorRef, tuple)) and (isinstance(z, _TensorRef) or (len(z) == 2 and z[0] in ("__dtype__",
                                                                                              "__device__")))),
                           pytree.tree_map(dec, kwargs), outs))
    feed_names = []
    for name, (vid, shape, dt) in model["feeds"].items():
        s = SymTensor(torch.empty(shape, dtype=convert_dtype(dt), device="meta"), prog, vid=vid, name=name)
        prog.feeds[name] = s
        prog.vars[vid] = s
        feed_names.append(name)
    fetch = []
    for vid in model["fetch"]:
        s = prog.vars.get(vid)
        if s is None:
            s = SymTensor(torch.empty(0, device="meta"), prog, vid=vid)
            prog.vars[vid] = s
        fetch.append(Tensor._wrap(s))
    return prog, feed_names, fetch


def deserialize_persistables(program, data, executor=None):
    from ..framework.io import load as _load

    return _load(_io.BytesIO(data))


def load_inference_model(path_prefix, executor=None, **kwargs):
    """-> [program, feed_target_names, fetch_targets] (reference API)."""
    from ..framework.io import load as _load
    from ..framework.place import current_torch_device

    dev = executor._device if executor is not None else current_torch_device()
    with open(path_prefix + ".pdmodel", "rb") as f:
        head = f.read(1)
    from . import pdmodel

    if pdmodel.is_program_desc(head):
        prog = pdmodel.load(path_prefix, dev)
        return [prog, prog.feed_names, prog.fetch_names]
    params = _load(path_prefix + ".pdiparams")
    params = {k: Tensor._wrap(v._t.to(dev)) for k, v in params.items()}
    with open(path_prefix + ".pdmodel", "rb") as f:
        data = f.read()
    prog, feeds, fetch = deserialize_program(data, params, dev)
    return [prog, feeds, fetch]


def save(program, model_path, protocol=4, **configs):
    from ..framework.io import save as _save

    _save({p.name: p for p in program.all_parameters()}, model_path + ".pdparams")


def load(program, model_path, executor=None, var_list=None):
    from ..framework.io import load as _load

    sd = _load(model_path + ".pdparams")
    set_program_state(program, sd)


def load_program_state(model_path, var_list=None):
    from ..framework.io import load as _load

    return _load(model_path + ".pdparams" if not model_path.endswith(".pdparams") else model_path)


def set_program_state(program, state_dict):
    for p in program.all_parameters():
        if p.name in state_dict:
            v = state_dict[p.name]
            with torch.no_grad():
                p._t.copy_(v._t if isinstance(v, Tensor) else torch.as_tensor(v))
