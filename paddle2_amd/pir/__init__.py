"""PIR — an SSA intermediate representation for static programs (reference: paddle/pir/ core IR —
Operation / Value / Block / Program, pd_op dialect, pass manager; python/paddle/pir/).

``translate_to_pir(program, feed_vars, fetch_vars)`` lowers a recorded static Program (static/graph.py) through
the Paddle-op lowering table (static/pdmodel.py) into SSA form: parameters become ``builtin.parameter`` ops,
feeds ``pd_op.data``, fetch targets ``pd_op.fetch``, everything else ``pd_op.<name>`` with typed result
Values (shape + dtype) and use lists.  ``run(program, feeds)`` interprets it with the framework's kernels (a
``pd_op.fused_gemm_epilogue`` produced by the fusion pass runs the Linear GEMM node + the fused bias-act
kernel).  Passes live in ``pir.passes``; primitive decomposition in ``paddle2_amd.decomposition``.
"""
from __future__ import annotations

import itertools

import torch

_ids = itertools.count()

# ProgramDesc op type -> PIR pd_op name
_DESC2PIR = {"matmul_v2": "matmul", "elementwise_add": "add", "elementwise_sub": "subtract",
             "elementwise_mul": "multiply", "elementwise_div": "divide", "reshape2": "reshape",
             "transpose2": "transpose", "flatten_contiguous_range": "flatten", "lookup_table_v2": "embedding",
             "reduce_mean": "mean", "reduce_sum": "sum", "reduce_max": "max", "hard_swish": "hardswish"}


class Value:
    def __init__(self, shape, dtype, op=None, index=0, name=None):
        self.id = next(_ids)
        self.shape = list(shape) if shape is not None else None
        self.dtype = dtype
        self._op = op
        self._index = index
        self.name = name
        self.uses = []  # (op, operand index)

    def get_defining_op(self):
        return self._op

    def use_empty(self):
        return not self.uses

    def replace_all_uses_with(self, other):
        for op, i in list(self.uses):
            op._operands[i] = other
            other.uses.append((op, i))
        self.uses = []

    def type_str(self):
        dt = {torch.float32: "f32", torch.float16: "f16", torch.bfloat16: "bf16", torch.int64: "i64",
              torch.int32: "i32", torch.bool: "b"}.get(self.dtype, str(self.dtype))
        shp = "x".join("?" if (s is None or s < 0) else str(s) for s in (self.shape or []))
        return f"tensor<{shp}x{dt}>" if shp else f"tensor<{dt}>"

    def __repr__(self):
        return f"%{self.id}"


class Operation:
    def __init__(self, name, operands, result_types, attrs=None):
        self._name = name
        self._operands = list(operands)
        self.attrs_ = dict(attrs or {})
        self._results = [Value(s, d, self, i) for i, (s, d) in enumerate(result_types)]
        self.block = None
        for i, v in enumerate(self._operands):
            v.uses.append((self, i))

    def name(self):
        return self._name

    def operands(self):
        return list(self._operands)

    def operand_source(self, i):
        return self._operands[i]

    def results(self):
        return list(self._results)

    def result(self, i):
        return self._results[i]

    def attrs(self):
        return dict(self.attrs_)

    def num_operands(self):
        return len(self._operands)

    def num_results(self):
        return len(self._results)

    def _drop_uses(self):
        for i, v in enumerate(self._operands):
            v.uses = [(o, j) for (o, j) in v.uses if not (o is self and j == i)]

    def __repr__(self):
        def fmt(v):
            if isinstance(v, bool):
                return "true" if v else "false"
            return repr(v)

        res = ", ".join(repr(r) for r in self._results)
        ops = ", ".join(repr(o) for o in self._operands)
        attrs = ",".join(f"{k}:{fmt(v)}" for k, v in self.attrs_.items() if k != "value" and not k.startswith("__"))
        tin = ", ".join(o.type_str() for o in self._operands)
        tout = ", ".join(r.type_str() for r in self._results)
        return f"({res}) = \"{self._name}\" ({ops}) {{{attrs}}} : ({tin}) -> {tout}"


class Block:
    def __init__(self):
        self.ops = []

    def append(self, op):
        op.block = self
        self.ops.append(op)
        return op

    def insert_before(self, anchor, op):
        op.block = self
        self.ops.insert(self.ops.index(anchor), op)
        return op

    def remove_op(self, op):
        op._drop_uses()
        self.ops.remove(op)


class Program:
    def __init__(self):
        self.block = Block()
        self.params = {}   # parameter value id -> tensor

    def global_block(self):
        return self.block

    def num_ops(self):
        return len(self.block.ops)

    def op_names(self):
        return [o.name() for o in self.block.ops]

    def __str__(self):
        return "{\n" + "\n".join("    " + repr(o) for o in self.block.ops) + "\n}"

    __repr__ = __str__


# ============================================================================================ translation
def _desc_attr_value(a):
    from ..static.pdmodel import _attr_value

    return _attr_value(a)


def translate_to_pir(program, feed_vars, fetch_vars):
    """Static Program (recorded) -> PIR Program."""
    from ..static import pdmodel
    from ..static.io import _fn_name, _prune
    from ..static.proto import VT

    fetch_ids = [f._t._vid for f in fetch_vars]
    feeds = {v._t._name: v._t for v in feed_vars}
    desc, params = pdmodel.lower_program(program, _prune(program, fetch_ids), feeds, fetch_ids, _fn_name)
    block = desc["blocks"][0]
    vt2torch = {v: k for k, v in pdmodel._TORCH2VT.items()}
    var_type = {}
    for v in block["vars"]:
        lt = v["type"].get("lod_tensor")
        if lt:
            t = lt["tensor"]
            var_type[v["name"]] = (t.get("dims", []), vt2torch.get(t.get("data_type"), torch.float32))
    prog = Program()
    env = {}
    for name, t in sorted(params.items()):
        op = prog.block.append(Operation("builtin.parameter", [], [(list(t.shape), t.dtype)], {"parameter_name": name}))
        env[name] = op.result(0)
        prog.params[op.result(0).id] = t
    fetch_names = []
    for d in block["ops"]:
        at = {a["name"]: _desc_attr_value(a) for a in d.get("attrs", [])}
        ins = {v["parameter"]: v.get("arguments", []) for v in d["inputs"]}
        outs = {v["parameter"]: v.get("arguments", []) for v in d["outputs"]}
        if d["type"] == "feed":
            name = outs["Out"][0]
            shp, dt = var_type[name]
            op = prog.block.append(Operation("pd_op.data", [], [(shp, dt)], {"name": name, "col": at.get("col", 0)}))
            env[name] = op.result(0)
            continue
        if d["type"] == "fetch":
            src = ins["X"][0]
            prog.block.append(Operation("pd_op.fetch", [env[src]], [(env[src].shape, env[src].dtype)],
                                        {"name": src, "col": at.get("col", 0)}))
            fetch_names.append(src)
            continue
        operands, slots = [], []
        for slot, names in ins.items():
            for n in names:
                operands.append(env[n])
                slots.append(slot)
        res_names = [(slot, n) for slot, names in outs.items() for n in names]
        rtypes = [var_type.get(n, (None, torch.float32)) for _, n in res_names]
        at["__slots__"] = slots
        at["__out_slots__"] = [s for s, _ in res_names]
        op = prog.block.append(Operation("pd_op." + _DESC2PIR.get(d["type"], d["type"]), operands, rtypes, at))
        for i, (_, n) in enumerate(res_names):
            env[n] = op.result(i)
    return prog


# ============================================================================================ interpreter
def _kernels(device=None):
    from ..ops import fused as FU
    from ..ops import torch_ops as T
    from ..static.pdmodel import PdProgram

    desc_name = {v: k for k, v in _DESC2PIR.items()}

    def via_desc(op, vals, at):
        """Run a translated op with the ProgramDesc interpreter's kernel (same Paddle semantics)."""
        name = op.name()[len("pd_op."):]
        ins = {}
        for s, v in zip(at.get("__slots__", []), vals):
            ins.setdefault(s, []).append(v)
        res = PdProgram._exec(None, desc_name.get(name, name), ins, at)
        slots = at.get("__out_slots__", ["Out"])
        return [res.get(s) for s in slots]

    F = torch.nn.functional
    prim = {
        "exp": lambda v, at: [torch.exp(v[0])],
        "log": lambda v, at: [torch.log(v[0])],
        "tanh": lambda v, at: [torch.tanh(v[0])],
        "erf": lambda v, at: [torch.erf(v[0])],
        "rsqrt": lambda v, at: [torch.rsqrt(v[0])],
        "sigmoid": lambda v, at: [torch.sigmoid(v[0])],
        "max": lambda v, at: [torch.amax(v[0], dim=at["axis"], keepdim=at.get("keepdim", True))],
        "sum": lambda v, at: [torch.sum(v[0], dim=at["axis"], keepdim=at.get("keepdim", True))]
        if "axis" in at else None,
        "full": lambda v, at: [torch.full(at["shape"], at["value"], dtype=at.get("dtype", torch.float32),
                                          device=device)],
        # primitives of decomposition.rules / decomposition.vjp
        "sqrt": lambda v, at: [torch.sqrt(v[0])],
        "abs": lambda v, at: [torch.abs(v[0])],
        "sign": lambda v, at: [torch.sign(v[0])],
        "floor": lambda v, at: [torch.floor(v[0])],
        "pow": lambda v, at: [torch.pow(v[0], at["y"])],
        "reshape": lambda v, at: [v[0].reshape(at["shape"])],
        "concat": lambda v, at: [torch.cat(v, dim=at["axis"])],
        "gather": lambda v, at: [torch.index_select(v[0], at["axis"], v[1].reshape(-1).long())],
        "take_along_axis": lambda v, at: [torch.take_along_dim(v[0], v[1].long(), dim=at["axis"])],
        "matmul": lambda v, at: [torch.matmul(v[0].mT if at.get("transpose_x") else v[0],
                                              v[1].mT if at.get("transpose_y") else v[1])],
        "cast": lambda v, at: [v[0].to(at["dtype"])],
        "where": lambda v, at: [torch.where(v[0], v[1], v[2])],
        "greater_than": lambda v, at: [torch.gt(v[0], v[1])],
        "greater_equal": lambda v, at: [torch.ge(v[0], v[1])],
        "less_than": lambda v, at: [torch.lt(v[0], v[1])],
        "less_equal": lambda v, at: [torch.le(v[0], v[1])],
        "equal": lambda v, at: [torch.eq(v[0], v[1])],
        "not_equal": lambda v, at: [torch.ne(v[0], v[1])],
        "arange": lambda v, at: [torch.arange(at["start"], at["end"], at["step"], dtype=at.get("dtype"),
                                              device=device)],
        "uniform": lambda v, at: [_uniform(at, device)],
        "expand": lambda v, at: [v[0].expand(at["shape"]).contiguous()],
        "transpose": lambda v, at: [v[0].permute(at["perm"])],
        "slice": lambda v, at: [v[0].narrow(at["axis"], at["start"], at["end"] - at["start"])],
        "index_add": lambda v, at: [torch.index_add(v[0], at["axis"], v[1].reshape(-1).long(), v[2])],
        "scatter_add_along": lambda v, at: [torch.scatter_add(v[0], at["axis"], v[1].long(), v[2])],
        "min": lambda v, at: [torch.amin(v[0], dim=at["axis"], keepdim=at.get("keepdim", True))],
    }

    def fused_gemm_epilogue(op, vals, at):
        x, w, b = vals[0], vals[1], vals[2]
        y = T.linear(x, w.t() if at.get("trans_y") else w)
        return [FU.bias_act(y, b, at.get("activation", "identity"))]

    return via_desc, prim, fused_gemm_epilogue


def _uniform(at, device):
    g = None
    if at.get("seed"):
        g = torch.Generator(device=device or "cpu").manual_seed(int(at["seed"]))
    return torch.rand(at["shape"], generator=g, device=device) * (at["max"] - at["min"]) + at["min"]


_BINARY_PRIM = {"pd_op.subtract": torch.sub, "pd_op.divide": torch.div, "pd_op.multiply": torch.mul,
                "pd_op.add": torch.add, "pd_op.maximum": torch.maximum, "pd_op.minimum": torch.minimum}


@torch.no_grad()
def run(program, feeds, device=None):
    """Execute a PIR Program: feeds in pd_op.data column order -> fetch values in pd_op.fetch column order
    (inference: no autograd graph)."""
    if device is None:
        for f in feeds:
            t = f._t if hasattr(f, "_t") else f
            if isinstance(t, torch.Tensor):
                device = t.device
                break
    via_desc, prim, fge = _kernels(device)
    env = {}
    out = {}
    for op in program.block.ops:
        n = op.name()
        if n == "builtin.parameter":
            t = program.params[op.result(0).id]
            env[op.result(0).id] = t.to(device) if device is not None else t
            continue
        if n == "pd_op.data":
            f = feeds[op.attrs_["col"]]
            env[op.result(0).id] = f._t if hasattr(f, "_t") else f
            continue
        vals = [env[v.id] for v in op.operands()]
        if n == "pd_op.fetch":
            out[op.attrs_["col"]] = vals[0]
            continue
        at = op.attrs_
        short = n[len("pd_op."):]
        if n == "pd_op.fused_gemm_epilogue":
            res = fge(op, vals, at)
        elif n in _BINARY_PRIM and "__slots__" not in at:
            res = [_BINARY_PRIM[n](vals[0], vals[1])]
        elif short in prim and "__slots__" not in at and (short != "sum" or "axis" in at):
            res = prim[short](vals, at)
        elif n == "pd_op.scale" and "__slots__" not in at:
            res = [vals[0] * at.get("scale", 1.0) + at.get("bias", 0.0)]
        else:
            res = via_desc(op, vals, at)
        for r, v in zip(op.results(), res):
            env[r.id] = v
    return [out[i] for i in sorted(out)]


from . import dialect, drr, passes, serialize  # noqa: E402,F401
from .dialect import IrContext, VerifyError, verify  # noqa: E402,F401
from .serialize import load, save  # noqa: E402,F401
