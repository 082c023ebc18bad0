"""Reference-format inference models: ``.pdmodel`` = a serialized ProgramDesc (framework.proto) with Paddle op
types, ``.pdiparams`` = the persistable tensors as consecutive LoDTensor records in name order (save_combine),
as written by the reference's ``paddle.jit.save`` / ``paddle.static.save_inference_model``
(python/paddle/static/io.py, paddle/fluid/operators/save_combine_op).

Export: the recorded Program (static/graph.py, torch-level ops) is lowered op by op to Paddle op types —
conv2d, pool2d, matmul_v2, elementwise_*, layer_norm, batch_norm, softmax, reshape2, transpose2, concat,
flatten_contiguous_range, lookup_table_v2, reduce_*, scale and the activations — with the reference's
input / output slot names and attributes.  ``lower_program`` raises ``Unmapped`` for an op outside that set (the
caller then keeps the framework's own program format).

Load: ``PdProgram`` interprets a ProgramDesc with the same op set (feed / fetch ops included), so a model
written here — or a reference-written model using those ops — runs on the MI355X through the framework's ops.
"""
from __future__ import annotations

import torch

from . import proto as P
from .graph import VarRef

_TORCH2VT = {torch.float32: P.VT["FP32"], torch.float16: P.VT["FP16"], torch.bfloat16: P.VT["BF16"],
             torch.float64: P.VT["FP64"], torch.int64: P.VT["INT64"], torch.int32: P.VT["INT32"],
             torch.int16: P.VT["INT16"], torch.int8: P.VT["INT8"], torch.uint8: P.VT["UINT8"], torch.bool: P.VT["BOOL"]}
_VT2TORCH = {v: k for k, v in _TORCH2VT.items()}


class Unmapped(Exception):
    pass


# ============================================================================================ attributes
def _attr(name, v):
    if isinstance(v, bool):
        return {"name": name, "type": P.AT["BOOLEAN"], "b": v}
    if isinstance(v, int):
        return ({"name": name, "type": P.AT["INT"], "i": v} if -2 ** 31 <= v < 2 ** 31
                else {"name": name, "type": P.AT["LONG"], "l": v})
    if isinstance(v, float):
        return {"name": name, "type": P.AT["FLOAT"], "f": v}
    if isinstance(v, str):
        return {"name": name, "type": P.AT["STRING"], "s": v}
    v = list(v)
    if all(isinstance(e, bool) for e in v) and v:
        return {"name": name, "type": P.AT["BOOLEANS"], "bools": v}
    if all(isinstance(e, int) for e in v):
        return {"name": name, "type": P.AT["INTS"], "ints": v}
    if all(isinstance(e, (int, float)) for e in v):
        return {"name": name, "type": P.AT["FLOATS"], "floats": [float(e) for e in v]}
    if all(isinstance(e, str) for e in v):
        return {"name": name, "type": P.AT["STRINGS"], "strings": v}
    raise Unmapped(f"attribute {name}={v!r}")


_ATTR_KEY = {0: "i", 1: "f", 2: "s", 3: "ints", 4: "floats", 5: "strings", 6: "b", 7: "bools", 8: "block_idx",
             9: "l", 10: "blocks_idx", 11: "longs", 12: "float64s", 13: "var_name", 14: "vars_name", 15: "float64"}


def _attr_value(a):
    t = a.get("type")
    v = a.get(_ATTR_KEY.get(t, "i"))
    if t == P.AT["BOOLEAN"]:
        return bool(v)
    if t == P.AT["BOOLEANS"]:
        return [bool(e) for e in v]
    return v


def _pair(v, n=2):
    return [int(e) for e in v] if isinstance(v, (list, tuple)) else [int(v)] * n


# ============================================================================================ lowering
class _Lowering:
    def __init__(self, program):
        self.program = program
        self.ops = []
        self.vars = {}       # name -> (dtype, shape, persistable)
        self.params = {}     # name -> tensor
        self._tid = {}
        self._tmp = 0

    def var_of(self, x):
        """Name of an op argument (VarRef / parameter / constant tensor)."""
        if isinstance(x, VarRef):
            name = self.names.get(x.vid) or f"tmp_{x.vid}"
            self.names[x.vid] = name
            meta = self.program.vars.get(x.vid)
            if meta is not None and name not in self.vars:
                self.vars[name] = (meta.dtype, list(meta.shape), False)
            return name
        if isinstance(x, torch.Tensor):
            key = id(x)
            if key not in self._tid:
                p = getattr(x, "_pd_param", None)
                nm = p.name if p is not None else f"const_{len(self._tid)}"
                self._tid[key] = nm
                self.params[nm] = x.detach()
                self.vars[nm] = (x.dtype, list(x.shape), True)
            return self._tid[key]
        raise Unmapped(f"argument {x!r}")

    def out(self, vid):
        name = self.names.get(vid) or f"tmp_{vid}"
        self.names[vid] = name
        meta = self.program.vars.get(vid)
        if meta is not None:
            self.vars[name] = (meta.dtype, list(meta.shape), False)
        return name

    def tmp(self, like):
        self._tmp += 1
        name = f"tmp_aux_{self._tmp}"
        self.vars[name] = (like[0], like[1], False)
        return name

    def emit(self, type_, inputs, outputs, **attrs):
        self.ops.append({"type": type_,
                         "inputs": [{"parameter": k, "arguments": v} for k, v in inputs.items()],
                         "outputs": [{"parameter": k, "arguments": v} for k, v in outputs.items()],
                         "attrs": [_attr(k, v) for k, v in attrs.items()]})

    # ---------------------------------------------------------------- op table
    def lower(self, name, args, kwargs, outs):
        o = self.out(outs[0]) if outs and outs[0] is not None else None
        meta = self.vars.get(o, (torch.float32, []))
        a = list(args)
        kw = dict(kwargs)
        unary = {"torch.nn.functional:relu": "relu", "torch:relu": "relu", "tensor:relu": "relu",
                 "torch:sigmoid": "sigmoid", "tensor:sigmoid": "sigmoid", "torch:tanh": "tanh", "tensor:tanh": "tanh",
                 "torch.nn.functional:silu": "silu", "torch:exp": "exp", "torch:sqrt": "sqrt",
                 "torch.nn.functional:hardswish": "hard_swish", "torch.nn.functional:relu6": "relu6"}
        if name in unary:
            self.emit(unary[name], {"X": [self.var_of(a[0])]}, {"Out": [o]})
        elif name in ("torch._C._nn:gelu", "torch.nn.functional:gelu"):
            self.emit("gelu", {"X": [self.var_of(a[0])]}, {"Out": [o]},
                      approximate=kw.get("approximate", "none") == "tanh")
        elif name == "torch:conv2d":
            x, w = a[0], a[1]
            b, stride, pad, dil, groups = (a + [None, 1, 0, 1, 1][len(a) - 2:])[2:7]
            algo = "EXPLICIT"
            if isinstance(pad, str):
                algo, pad = pad.upper(), 0
            target = o if b is None else self.tmp(meta)
            self.emit("conv2d", {"Input": [self.var_of(x)], "Filter": [self.var_of(w)]}, {"Output": [target]},
                      strides=_pair(stride), paddings=_pair(pad), dilations=_pair(dil), groups=int(groups),
                      padding_algorithm=algo, data_format="NCHW")
            if b is not None:
                self.emit("elementwise_add", {"X": [target], "Y": [self.var_of(b)]}, {"Out": [o]}, axis=1)
        elif name in ("torch.nn.functional:max_pool2d", "torch.nn.functional:avg_pool2d"):
            ks = _pair(a[1] if len(a) > 1 else kw["kernel_size"])
            st = a[2] if len(a) > 2 else kw.get("stride")
            st = ks if st is None or st == [] else _pair(st)
            pad = _pair(a[3] if len(a) > 3 else kw.get("padding", 0))
            ceil = bool(kw.get("ceil_mode", False))
            if name.endswith("max_pool2d"):
                if _pair(kw.get("dilation", 1)) != [1, 1] or kw.get("return_indices"):
                    raise Unmapped("max_pool2d dilation / indices")
                self.emit("pool2d", {"X": [self.var_of(a[0])]}, {"Out": [o]}, pooling_type="max", ksize=ks,
                          strides=st, paddings=pad, ceil_mode=ceil, global_pooling=False, adaptive=False,
                          exclusive=True, data_format="NCHW", padding_algorithm="EXPLICIT")
            else:
                self.emit("pool2d", {"X": [self.var_of(a[0])]}, {"Out": [o]}, pooling_type="avg", ksize=ks,
                          strides=st, paddings=pad, ceil_mode=ceil, global_pooling=False, adaptive=False,
                          exclusive=not kw.get("count_include_pad", True), data_format="NCHW",
                          padding_algorithm="EXPLICIT")
        elif name in ("torch.nn.functional:adaptive_avg_pool2d", "torch._C._nn:adaptive_avg_pool2d"):
            self.emit("pool2d", {"X": [self.var_of(a[0])]}, {"Out": [o]}, pooling_type="avg",
                      ksize=_pair(a[1] if len(a) > 1 else kw["output_size"]), strides=[1, 1], paddings=[0, 0],
                      ceil_mode=False, global_pooling=False, adaptive=True, exclusive=True, data_format="NCHW",
                      padding_algorithm="EXPLICIT")
        elif name in ("torch:flatten", "tensor:flatten"):
            s = a[1] if len(a) > 1 else kw.get("start_dim", 0)
            e = a[2] if len(a) > 2 else kw.get("end_dim", -1)
            self.emit("flatten_contiguous_range", {"X": [self.var_of(a[0])]}, {"Out": [o]}, start_axis=int(s),
                      stop_axis=int(e))
        elif name == "torch:addmm":
            mm = self.tmp(meta)
            self.emit("matmul_v2", {"X": [self.var_of(a[1])], "Y": [self.var_of(a[2])]}, {"Out": [mm]},
                      trans_x=False, trans_y=False)
            self.emit("elementwise_add", {"X": [mm], "Y": [self.var_of(a[0])]}, {"Out": [o]}, axis=-1)
        elif name == "torch.nn.functional:linear":
            b = a[2] if len(a) > 2 else kw.get("bias")
            mm = o if b is None else self.tmp(meta)
            self.emit("matmul_v2", {"X": [self.var_of(a[0])], "Y": [self.var_of(a[1])]}, {"Out": [mm]},
                      trans_x=False, trans_y=True)
            if b is not None:
                self.emit("elementwise_add", {"X": [mm], "Y": [self.var_of(b)]}, {"Out": [o]}, axis=-1)
        elif name in ("torch:matmul", "tensor:matmul", "torch:mm", "tensor:__matmul__", "torch:bmm"):
            self.emit("matmul_v2", {"X": [self.var_of(a[0])], "Y": [self.var_of(a[1])]}, {"Out": [o]},
                      trans_x=False, trans_y=False)
        elif name.endswith(":layer_norm"):
            x, w, b = a[0], a[1], a[2]
            eps = a[3] if len(a) > 3 else kw.get("eps", kw.get("epsilon", 1e-5))
            xm = self.vars[self.var_of(x)]
            nd = len(w.shape) if isinstance(w, torch.Tensor) else 1
            mean, var = self.tmp((torch.float32, [])), self.tmp((torch.float32, []))
            self.emit("layer_norm", {"X": [self.var_of(x)], "Scale": [self.var_of(w)], "Bias": [self.var_of(b)]},
                      {"Y": [o], "Mean": [mean], "Variance": [var]}, epsilon=float(eps),
                      begin_norm_axis=len(xm[1]) - nd)
        elif name in ("torch:softmax", "torch.nn.functional:softmax", "tensor:softmax"):
            dim = a[1] if len(a) > 1 else kw.get("dim", -1)
            self.emit("softmax", {"X": [self.var_of(a[0])]}, {"Out": [o]}, axis=int(dim))
        elif name in ("torch:add", "tensor:add", "tensor:__add__", "torch:sub", "tensor:sub", "tensor:__sub__",
                      "torch:mul", "tensor:mul", "tensor:__mul__", "torch:div", "tensor:div", "tensor:__truediv__"):
            kind = {"add": "add", "sub": "sub", "mul": "mul", "div": "div", "__add__": "add", "__sub__": "sub",
                    "__mul__": "mul", "__truediv__": "div"}[name.split(":")[1]]
            x, y = a[0], a[1]
            if isinstance(y, (int, float)):
                sc, bias = {"add": (1.0, float(y)), "sub": (1.0, -float(y)), "mul": (float(y), 0.0),
                            "div": (1.0 / float(y), 0.0)}[kind]
                self.emit("scale", {"X": [self.var_of(x)]}, {"Out": [o]}, scale=sc, bias=bias, bias_after_scale=True)
            else:
                self.emit(f"elementwise_{kind}", {"X": [self.var_of(x)], "Y": [self.var_of(y)]}, {"Out": [o]},
                          axis=-1)
        elif name in ("tensor:reshape", "torch:reshape", "tensor:view"):
            shp = a[1:] if len(a) > 2 else a[1]
            shp = [int(s) for s in (shp if isinstance(shp, (list, tuple)) else [shp])]
            xs = self.tmp((torch.int64, []))
            self.emit("reshape2", {"X": [self.var_of(a[0])]}, {"Out": [o], "XShape": [xs]}, shape=shp)
        elif name in ("tensor:permute", "torch:permute"):
            perm = a[1:] if len(a) > 2 else a[1]
            xs = self.tmp((torch.int64, []))
            self.emit("transpose2", {"X": [self.var_of(a[0])]}, {"Out": [o], "XShape": [xs]},
                      axis=[int(p) for p in perm])
        elif name in ("torch:transpose", "tensor:transpose"):
            nd = len(self.vars[self.var_of(a[0])][1])
            perm = list(range(nd))
            d0, d1 = a[1] % nd, a[2] % nd
            perm[d0], perm[d1] = perm[d1], perm[d0]
            xs = self.tmp((torch.int64, []))
            self.emit("transpose2", {"X": [self.var_of(a[0])]}, {"Out": [o], "XShape": [xs]}, axis=perm)
        elif name in ("torch:cat", "torch:concat"):
            dim = a[1] if len(a) > 1 else kw.get("dim", 0)
            self.emit("concat", {"X": [self.var_of(t) for t in a[0]]}, {"Out": [o]}, axis=int(dim))
        elif name == "torch.nn.functional:batch_norm":
            x, rm, rv = a[0], a[1], a[2]
            w = a[3] if len(a) > 3 else kw.get("weight")
            b = a[4] if len(a) > 4 else kw.get("bias")
            training = a[5] if len(a) > 5 else kw.get("training", False)
            mom = a[6] if len(a) > 6 else kw.get("momentum", 0.1)
            eps = a[7] if len(a) > 7 else kw.get("eps", 1e-5)
            if training or w is None or b is None:
                raise Unmapped("batch_norm in training mode / without affine")
            outs_ = {"Y": [o]}
            for slot in ("MeanOut", "VarianceOut", "SavedMean", "SavedVariance"):
                outs_[slot] = [self.tmp((torch.float32, []))]
            self.emit("batch_norm", {"X": [self.var_of(x)], "Scale": [self.var_of(w)], "Bias": [self.var_of(b)],
                                     "Mean": [self.var_of(rm)], "Variance": [self.var_of(rv)]}, outs_,
                      epsilon=float(eps), momentum=1.0 - float(mom), is_test=True, data_layout="NCHW",
                      use_global_stats=True)
        elif name in ("torch:mean", "tensor:mean", "torch:sum", "tensor:sum"):
            dim = a[1] if len(a) > 1 else kw.get("dim")
            keep = bool(a[2] if len(a) > 2 else kw.get("keepdim", False))
            op = "reduce_mean" if "mean" in name else "reduce_sum"
            dims = [] if dim is None else ([int(dim)] if isinstance(dim, int) else [int(d) for d in dim])
            self.emit(op, {"X": [self.var_of(a[0])]}, {"Out": [o]}, dim=dims, keep_dim=keep, reduce_all=dim is None)
        elif name == "torch.nn.functional:embedding":
            pad = kw.get("padding_idx", a[2] if len(a) > 2 else None)
            self.emit("lookup_table_v2", {"Ids": [self.var_of(a[0])], "W": [self.var_of(a[1])]}, {"Out": [o]},
                      padding_idx=-1 if pad is None else int(pad))
        elif name in ("torch.nn.functional:dropout", "tensor:contiguous", "tensor:clone"):
            self.emit("scale", {"X": [self.var_of(a[0])]}, {"Out": [o]}, scale=1.0, bias=0.0, bias_after_scale=True)
        else:
            raise Unmapped(name)


def lower_program(program, ops, feeds, fetch_ids, fn_name):
    """-> (ProgramDesc dict, {param name: tensor}); raises Unmapped for an op outside the table."""
    L = _Lowering(program)
    L.names = {}
    feed_names = []
    for nm, s in feeds.items():
        L.names[s._vid] = nm
        L.vars[nm] = (s.dtype, list(s.shape), False)
        feed_names.append(nm)
    body = L.ops
    for op in ops:
        L.lower(fn_name(op.fn), op.args, op.kwargs, op.outs)
    fetch_names = [L.names.get(v) or f"tmp_{v}" for v in fetch_ids]
    feed_ops = [{"type": "feed", "inputs": [{"parameter": "X", "arguments": ["feed"]}],
                 "outputs": [{"parameter": "Out", "arguments": [n]}], "attrs": [_attr("col", i)]}
                for i, n in enumerate(feed_names)]
    fetch_ops = [{"type": "fetch", "inputs": [{"parameter": "X", "arguments": [n]}],
                  "outputs": [{"parameter": "Out", "arguments": ["fetch"]}], "attrs": [_attr("col", i)]}
                 for i, n in enumerate(fetch_names)]
    vars_ = [{"name": "feed", "type": {"type": P.VT["FEED_MINIBATCH"]}, "persistable": True},
             {"name": "fetch", "type": {"type": P.VT["FETCH_LIST"]}, "persistable": True}]
    for nm, (dt, shape, pers) in L.vars.items():
        dims = [-1 if (nm in feed_names and i == 0) else int(d) for i, d in enumerate(shape)]
        vars_.append({"name": nm, "persistable": pers, "is_parameter": pers, "stop_gradient": True,
                      "need_check_feed": nm in feed_names,
                      "type": {"type": P.VT["LOD_TENSOR"],
                               "lod_tensor": {"tensor": {"data_type": _TORCH2VT.get(dt, P.VT["FP32"]),
                                                         "dims": dims}}}})
    block = {"idx": 0, "parent_idx": -1, "vars": vars_, "ops": feed_ops + body + fetch_ops, "forward_block_idx": -1}
    desc = {"blocks": [block], "version": {"version": 0}}
    return desc, L.params


# ============================================================================================ .pdiparams
def _raw(t):
    t = t.detach().cpu().contiguous()
    if t.dtype == torch.bfloat16:
        return t.view(torch.int16).numpy().tobytes()
    return t.numpy().tobytes()


def save_params(path, params):
    """save_combine layout: every persistable in sorted-name order."""
    with open(path, "wb") as f:
        for nm in sorted(params):
            t = params[nm]
            P.write_lod_tensor(f, _TORCH2VT[t.dtype], list(t.shape), _raw(t))


def load_params(path, names):
    out = {}
    with open(path, "rb") as f:
        for nm in names:
            rec = P.read_lod_tensor(f)
            if rec is None:
                raise ValueError(f"{path}: ran out of tensors at {nm}")
            dt, dims, raw, _ = rec
            tdt = _VT2TORCH[dt]
            if tdt == torch.bfloat16:
                arr = torch.frombuffer(bytearray(raw), dtype=torch.int16).view(torch.bfloat16)
            else:
                arr = torch.frombuffer(bytearray(raw), dtype=tdt) if raw else torch.empty(0, dtype=tdt)
            out[nm] = arr.reshape([int(d) for d in dims]).clone()
    return out


def is_program_desc(data):
    """ProgramDesc bytes start with field 1 (blocks, length-delimited) -> 0x0a; the framework's own format is a
    pickle (0x80)."""
    return len(data) > 0 and data[0] == 0x0A


# ============================================================================================ interpreter
def _bcast(x, y, axis):
    """Paddle elementwise broadcast: y's dims align with x's starting at ``axis`` (-1: trailing)."""
    if axis == -1 or y.dim() == x.dim() or y.dim() == 0:
        return y
    shape = [1] * axis + list(y.shape) + [1] * (x.dim() - axis - y.dim())
    return y.reshape(shape)


def _pool2d(x, at):
    ks, st, pad = at["ksize"], at.get("strides", [1, 1]), at.get("paddings", [0, 0])
    if len(pad) == 4:
        pad = [pad[0], pad[2]]
    if at.get("global_pooling"):
        ks, pad = list(x.shape[2:]), [0, 0]
    F = torch.nn.functional
    if at.get("adaptive"):
        return (F.adaptive_max_pool2d if at["pooling_type"] == "max" else F.adaptive_avg_pool2d)(x, ks)
    if at["pooling_type"] == "max":
        return F.max_pool2d(x, ks, st, pad, ceil_mode=at.get("ceil_mode", False))
    return F.avg_pool2d(x, ks, st, pad, ceil_mode=at.get("ceil_mode", False),
                        count_include_pad=not at.get("exclusive", True))


class PdProgram:
    """Runs a decoded ProgramDesc block 0 with torch ops (the framework's kernels where they exist)."""

    def __init__(self, desc, params, device=None):
        self.desc = desc
        self.block = desc["blocks"][0]
        self.device = device
        self.params = {k: (v.to(device) if device is not None else v) for k, v in params.items()}
        self.feed_names = [self._io(o, "Out")[0] for o in self.block["ops"] if o["type"] == "feed"]
        self.fetch_names = [self._io(o, "X", True)[0] for o in self.block["ops"] if o["type"] == "fetch"]

    @staticmethod
    def _io(op, slot, inputs=False):
        for v in op["inputs" if inputs else "outputs"]:
            if v["parameter"] == slot:
                return v.get("arguments", [])
        return []

    def run(self, feeds):
        env = dict(self.params)
        fetched = {}
        for op in self.block["ops"]:
            at = {a["name"]: _attr_value(a) for a in op.get("attrs", [])}
            ins = {v["parameter"]: [env.get(n) for n in v.get("arguments", [])] for v in op["inputs"]}
            outs = {v["parameter"]: v.get("arguments", []) for v in op["outputs"]}
            t = op["type"]
            if t == "feed":
                x = feeds[at.get("col", 0)]
                env[outs["Out"][0]] = x
                continue
            if t == "fetch":
                fetched[at.get("col", 0)] = ins["X"][0]
                continue
            res = self._exec(t, ins, at)
            for slot, val in res.items():
                if slot in outs and outs[slot]:
                    env[outs[slot][0]] = val
        return [fetched[i] for i in sorted(fetched)]

    def _exec(self, t, ins, at):
        F = torch.nn.functional
        X = ins.get("X", [None])[0]
        act = {"relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh, "silu": F.silu, "exp": torch.exp,
               "sqrt": torch.sqrt, "hard_swish": F.hardswish, "relu6": F.relu6}
        if t in act:
            return {"Out": act[t](X)}
        if t == "gelu":
            return {"Out": F.gelu(X, approximate="tanh" if at.get("approximate") else "none")}
        if t in ("conv2d", "depthwise_conv2d"):
            x, w = ins["Input"][0], ins["Filter"][0]
            pad = at.get("paddings", [0, 0])
            algo = at.get("padding_algorithm", "EXPLICIT")
            if algo in ("SAME", "VALID"):
                pad = algo.lower()
            elif len(pad) == 4:
                if pad[0] != pad[1] or pad[2] != pad[3]:
                    x = F.pad(x, [pad[2], pad[3], pad[0], pad[1]])
                    pad = [0, 0]
                else:
                    pad = [pad[0], pad[2]]
            nhwc = at.get("data_format", "NCHW") == "NHWC"
            if nhwc:
                x = x.permute(0, 3, 1, 2)
            y = F.conv2d(x, w, None, at.get("strides", [1, 1]), pad, at.get("dilations", [1, 1]), at.get("groups", 1))
            return {"Output": y.permute(0, 2, 3, 1) if nhwc else y}
        if t == "pool2d":
            return {"Out": _pool2d(X, at)}
        if t == "flatten_contiguous_range":
            return {"Out": torch.flatten(X, at.get("start_axis", 1), at.get("stop_axis", -1))}
        if t in ("matmul_v2", "matmul"):
            x, y = X, ins["Y"][0]
            if at.get("trans_x", at.get("transpose_X", False)):
                x = x.transpose(-1, -2)
            if at.get("trans_y", at.get("transpose_Y", False)):
                y = y.transpose(-1, -2)
            out = torch.matmul(x, y)
            if t == "matmul" and at.get("alpha", 1.0) != 1.0:
                out = out * at["alpha"]
            return {"Out": out}
        if t.startswith("elementwise_"):
            y = _bcast(X, ins["Y"][0], at.get("axis", -1))
            fn = {"add": torch.add, "sub": torch.sub, "mul": torch.mul, "div": torch.div, "max": torch.maximum,
                  "min": torch.minimum, "pow": torch.pow}[t.split("_", 1)[1]]
            return {"Out": fn(X, y)}
        if t == "scale":
            s, b = float(at.get("scale", 1.0)), float(at.get("bias", 0.0))
            return {"Out": X * s + b if at.get("bias_after_scale", True) else (X + b) * s}
        if t == "layer_norm":
            ax = at.get("begin_norm_axis", 1)
            shp = list(X.shape[ax:])
            sc = ins.get("Scale", [None])[0]
            bi = ins.get("Bias", [None])[0]
            y = F.layer_norm(X, shp, None if sc is None else sc.reshape(shp), None if bi is None else bi.reshape(shp),
                             at.get("epsilon", 1e-5))
            return {"Y": y}
        if t == "batch_norm":
            nhwc = at.get("data_layout", "NCHW") == "NHWC"
            x = X.permute(0, 3, 1, 2) if nhwc else X
            y = F.batch_norm(x, ins["Mean"][0], ins["Variance"][0], ins["Scale"][0], ins["Bias"][0], False, 0.0,
                             at.get("epsilon", 1e-5))
            return {"Y": y.permute(0, 2, 3, 1) if nhwc else y}
        if t == "softmax":
            return {"Out": torch.softmax(X, at.get("axis", -1))}
        if t in ("reshape2", "reshape"):
            shp = [X.shape[i] if s == 0 else s for i, s in enumerate(at["shape"])]
            return {"Out": X.reshape(shp)}
        if t in ("transpose2", "transpose"):
            return {"Out": X.permute(at["axis"])}
        if t == "concat":
            return {"Out": torch.cat(ins["X"], at.get("axis", 0))}
        if t in ("reduce_mean", "reduce_sum", "reduce_max"):
            fn = {"reduce_mean": torch.mean, "reduce_sum": torch.sum, "reduce_max": torch.amax}[t]
            if at.get("reduce_all") or not at.get("dim"):
                out = fn(X) if t != "reduce_max" else X.max()
                return {"Out": out.reshape([1] * X.dim()) if at.get("keep_dim") else out}
            return {"Out": fn(X, dim=at["dim"], keepdim=at.get("keep_dim", False))}
        if t == "lookup_table_v2":
            pad = at.get("padding_idx", -1)
            return {"Out": F.embedding(ins["Ids"][0], ins["W"][0], None if pad == -1 else pad)}
        if t == "dropout":
            if at.get("dropout_implementation", "downgrade_in_infer") == "downgrade_in_infer":
                return {"Out": X * (1.0 - at.get("dropout_prob", 0.5))}
            return {"Out": X}
        raise NotImplementedError(f"PdProgram: op {t!r} is not supported by the interpreter")


def program_param_names(desc):
    """Persistable (non feed / fetch) variable names in save_combine (sorted) order."""
    b = desc["blocks"][0]
    return sorted(v["name"] for v in b["vars"] if v.get("persistable")
                  and v["type"]["type"] not in (P.VT["FEED_MINIBATCH"], P.VT["FETCH_LIST"]))


def save(path_prefix, program, ops, feeds, fetch_ids, fn_name):
    desc, params = lower_program(program, ops, feeds, fetch_ids, fn_name)
    with open(path_prefix + ".pdmodel", "wb") as f:
        f.write(P.encode(desc, "ProgramDesc"))
    save_params(path_prefix + ".pdiparams", params)
    return desc


def load(path_prefix, device=None):
    with open(path_prefix + ".pdmodel", "rb") as f:
        desc = P.decode(f.read(), "ProgramDesc")
    params = load_params(path_prefix + ".pdiparams", program_param_names(desc))
    return PdProgram(desc, params, device)
