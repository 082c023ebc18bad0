"""ONNX export from the framework's own recorded Program (reference python/paddle/onnx/export.py, which drives
paddle2onnx over a ProgramDesc).

The Layer is recorded into a static Program (the same recording ``jit.save`` uses), every recorded op is mapped
to ONNX opset-17 nodes, parameters become initializers (raw little-endian data), and the ModelProto is written
with the framework's own protobuf wire codec (``static/proto.py``) over an ONNX schema table — no ``onnx`` or
``torch.onnx`` dependency (neither is usable in this image).  ``load_model_dict`` decodes a written file back to
plain dicts, and ``run_reference`` evaluates a decoded graph with numpy (the test oracle).
"""
from __future__ import annotations

import math
import os

import numpy as np
import torch
import torch.utils._pytree as pytree

from ..static import proto as P

P.SCHEMA.update({
    "onnx.OperatorSetIdProto": {1: ("domain", "string", False, None), 2: ("version", "varint", False, None)},
    "onnx.Dimension": {1: ("dim_value", "varint", False, None), 2: ("dim_param", "string", False, None)},
    "onnx.TensorShapeProto": {1: ("dim", "msg", True, "onnx.Dimension")},
    "onnx.TypeProto.Tensor": {1: ("elem_type", "varint", False, None), 2: ("shape", "msg", False, "onnx.TensorShapeProto")},
    "onnx.TypeProto": {1: ("tensor_type", "msg", False, "onnx.TypeProto.Tensor")},
    "onnx.ValueInfoProto": {1: ("name", "string", False, None), 2: ("type", "msg", False, "onnx.TypeProto"),
                            3: ("doc_string", "string", False, None)},
    "onnx.TensorProto": {1: ("dims", "varint", True, None), 2: ("data_type", "varint", False, None),
                         8: ("name", "string", False, None), 9: ("raw_data", "bytes", False, None)},
    "onnx.AttributeProto": {1: ("name", "string", False, None), 2: ("f", "float", False, None),
                            3: ("i", "varint", False, None), 4: ("s", "bytes", False, None),
                            5: ("t", "msg", False, "onnx.TensorProto"), 7: ("floats", "float", True, None),
                            8: ("ints", "varint", True, None), 20: ("type", "varint", False, None)},
    "onnx.NodeProto": {1: ("input", "string", True, None), 2: ("output", "string", True, None),
                       3: ("name", "string", False, None), 4: ("op_type", "string", False, None),
                       5: ("attribute", "msg", True, "onnx.AttributeProto"), 7: ("domain", "string", False, None)},
    "onnx.GraphProto": {1: ("node", "msg", True, "onnx.NodeProto"), 2: ("name", "string", False, None),
                        5: ("initializer", "msg", True, "onnx.TensorProto"),
                        11: ("input", "msg", True, "onnx.ValueInfoProto"),
                        12: ("output", "msg", True, "onnx.ValueInfoProto")},
    "onnx.ModelProto": {1: ("ir_version", "varint", False, None), 2: ("producer_name", "string", False, None),
                        3: ("producer_version", "string", False, None), 7: ("graph", "msg", False, "onnx.GraphProto"),
                        8: ("opset_import", "msg", True, "onnx.OperatorSetIdProto")},
})
P._BY_NAME.update({m: {v[0]: (k,) + v[1:] for k, v in f.items()} for m, f in P.SCHEMA.items() if m.startswith("onnx.")})

OPSET = 17
_DT = {torch.float32: 1, torch.uint8: 2, torch.int8: 3, torch.int16: 5, torch.int32: 6, torch.int64: 7,
       torch.bool: 9, torch.float16: 10, torch.float64: 11, torch.bfloat16: 16}
_NP = {1: np.float32, 2: np.uint8, 3: np.int8, 5: np.int16, 6: np.int32, 7: np.int64, 9: np.bool_, 10: np.float16,
       11: np.float64}


def _attr(name, v):
    if isinstance(v, float):
        return {"name": name, "f": v, "type": 1}
    if isinstance(v, bool) or isinstance(v, int):
        return {"name": name, "i": int(v), "type": 2}
    if isinstance(v, str):
        return {"name": name, "s": v.encode(), "type": 3}
    if isinstance(v, (list, tuple)) and all(isinstance(x, float) for x in v) and v:
        return {"name": name, "floats": list(v), "type": 6}
    return {"name": name, "ints": [int(x) for x in v], "type": 7}


def _tensor(name, t):
    t = t.detach().cpu()
    if t.dtype == torch.bfloat16:
        t = t.float()
    return {"name": name, "dims": list(t.shape), "data_type": _DT[t.dtype],
            "raw_data": t.contiguous().numpy().tobytes()}


def _value_info(name, shape, dtype):
    dt = _DT.get(dtype, 1) if dtype != torch.bfloat16 else 1
    return {"name": name, "type": {"tensor_type": {"elem_type": dt,
                                                   "shape": {"dim": [{"dim_value": int(d)} for d in shape]}}}}


class _Builder:
    def __init__(self, program):
        self.prog = program
        self.nodes, self.inits = [], []
        self.names = {}          # tensor key -> onnx value name
        self.k = 0

    def fresh(self, base="t"):
        self.k += 1
        return f"{base}_{self.k}"

    def node(self, op, inputs, outputs=None, **attrs):
        outputs = outputs or [self.fresh(op.lower())]
        self.nodes.append({"op_type": op, "input": list(inputs), "output": list(outputs), "name": self.fresh("n"),
                           "attribute": [_attr(k, v) for k, v in attrs.items()]})
        return outputs[0] if len(outputs) == 1 else outputs

    def const(self, value, dtype=torch.float32, name=None):
        n = name or self.fresh("c")
        self.inits.append(_tensor(n, torch.as_tensor(value, dtype=dtype)))
        return n

    def val(self, x):
        from ..static.graph import VarRef

        if isinstance(x, VarRef):
            return self.names[("v", x.vid)]
        if isinstance(x, torch.Tensor):
            key = ("p", id(x))
            if key not in self.names:
                p = getattr(x, "_pd_param", None)
                nm = (getattr(p, "name", None) or self.fresh("w")) if p is not None else self.fresh("const")
                self.inits.append(_tensor(nm, x))
                self.names[key] = nm
            return self.names[key]
        return self.const(x)

    def shape(self, x):
        from ..static.graph import VarRef

        return list(self.prog.vars[x.vid].shape) if isinstance(x, VarRef) else list(torch.as_tensor(x).shape)


def _key(op):
    import torch.nn.functional as F

    if op.fn is F.max_pool2d:
        return "max_pool2d"
    if op.fn is F.avg_pool2d:
        return "avg_pool2d"
    if op.fn is F.adaptive_avg_pool2d:
        return "adaptive_avg_pool2d"
    return op.name.rsplit(".", 1)[-1].lower()


def _pair(v):
    return list(v) if isinstance(v, (list, tuple)) else [int(v), int(v)]


def _convert(b, op):
    """Emit nodes for one recorded op; returns the list of output value names."""
    k = _key(op)
    a, kw = list(op.args), dict(op.kwargs)
    V = b.val
    if k == "addmm":
        return [b.node("Gemm", [V(a[1]), V(a[2]), V(a[0])])]
    if k in ("mm", "matmul", "bmm"):
        return [b.node("MatMul", [V(a[0]), V(a[1])])]
    if k == "linear":
        wt = b.node("Transpose", [V(a[1])], perm=[1, 0])
        y = b.node("MatMul", [V(a[0]), wt])
        return [b.node("Add", [y, V(a[2])]) if len(a) > 2 and a[2] is not None else y]
    binop = {"add": "Add", "sub": "Sub", "mul": "Mul", "div": "Div", "true_divide": "Div", "pow": "Pow",
             "maximum": "Max", "minimum": "Min"}
    if k in binop:
        x, y = a[0], a[1]
        alpha = kw.get("alpha", 1)
        yv = V(y) if not isinstance(y, (int, float)) else b.const(float(y))
        if alpha != 1:
            yv = b.node("Mul", [yv, b.const(float(alpha))])
        xv = V(x) if not isinstance(x, (int, float)) else b.const(float(x))
        return [b.node(binop[k], [xv, yv])]
    unop = {"relu": "Relu", "sigmoid": "Sigmoid", "tanh": "Tanh", "exp": "Exp", "log": "Log", "neg": "Neg",
            "sqrt": "Sqrt", "abs": "Abs", "erf": "Erf", "rsqrt": None, "dropout": "Identity", "clone": "Identity",
            "contiguous": "Identity", "flatten": None}
    if k in ("relu", "sigmoid", "tanh", "exp", "log", "neg", "sqrt", "abs", "erf", "dropout", "clone", "contiguous"):
        return [b.node(unop[k], [V(a[0])])]
    if k == "rsqrt":
        return [b.node("Reciprocal", [b.node("Sqrt", [V(a[0])])])]
    if k == "silu":
        x = V(a[0])
        return [b.node("Mul", [x, b.node("Sigmoid", [x])])]
    if k == "gelu":
        x = V(a[0])
        if kw.get("approximate", "none") == "tanh":
            inner = b.node("Mul", [b.const(math.sqrt(2 / math.pi)),
                                   b.node("Add", [x, b.node("Mul", [b.const(0.044715),
                                                                    b.node("Pow", [x, b.const(3.0)])])])])
            t = b.node("Tanh", [inner])
        else:
            t = b.node("Erf", [b.node("Div", [x, b.const(math.sqrt(2.0))])])
        return [b.node("Mul", [b.node("Mul", [x, b.const(0.5)]), b.node("Add", [t, b.const(1.0)])])]
    if k in ("softmax", "log_softmax", "_softmax"):
        axis = a[1] if len(a) > 1 and isinstance(a[1], int) else kw.get("dim", -1)
        return [b.node("Softmax" if k != "log_softmax" else "LogSoftmax", [V(a[0])], axis=int(axis))]
    if k in ("mean", "sum"):
        nd = len(b.shape(a[0]))
        dim = a[1] if len(a) > 1 and not isinstance(a[1], bool) else kw.get("dim")
        keep = bool(kw.get("keepdim", a[2] if len(a) > 2 and isinstance(a[2], bool) else False))
        axes = list(range(nd)) if dim is None else ([dim] if isinstance(dim, int) else list(dim))
        axes = [d % nd for d in axes]
        if k == "mean":
            return [b.node("ReduceMean", [V(a[0])], axes=axes, keepdims=int(keep))]
        return [b.node("ReduceSum", [V(a[0]), b.const(axes, torch.int64)], keepdims=int(keep))]
    if k in ("reshape", "view"):
        shape = list(a[1]) if isinstance(a[1], (list, tuple, torch.Size)) else [int(s) for s in a[1:]]
        return [b.node("Reshape", [V(a[0]), b.const(shape, torch.int64)])]
    if k in ("transpose", "permute", "movedim"):
        nd = len(b.shape(a[0]))
        if k == "permute":
            perm = list(a[1]) if isinstance(a[1], (list, tuple)) else list(a[1:])
        elif k == "transpose":
            perm = list(range(nd))
            i, j = a[1] % nd, a[2] % nd
            perm[i], perm[j] = perm[j], perm[i]
        else:
            src, dst = a[1] % nd, a[2] % nd
            rest = [d for d in range(nd) if d != src]
            rest.insert(dst, src)
            perm = rest
        return [b.node("Transpose", [V(a[0])], perm=[p % nd for p in perm])]
    if k == "flatten":
        nd = len(b.shape(a[0]))
        start = (a[1] if len(a) > 1 else kw.get("start_dim", 0)) % nd
        end = (a[2] if len(a) > 2 else kw.get("end_dim", -1)) % nd
        shp = b.shape(a[0])
        new = shp[:start] + [int(np.prod(shp[start:end + 1]))] + shp[end + 1:]
        return [b.node("Reshape", [V(a[0]), b.const(new, torch.int64)])]
    if k == "conv2d":
        x, w = a[0], a[1]
        bias = a[2] if len(a) > 2 else kw.get("bias")
        stride = _pair(a[3] if len(a) > 3 else kw.get("stride", 1))
        pad = _pair(a[4] if len(a) > 4 else kw.get("padding", 0))
        dil = _pair(a[5] if len(a) > 5 else kw.get("dilation", 1))
        groups = a[6] if len(a) > 6 else kw.get("groups", 1)
        ins = [V(x), V(w)] + ([V(bias)] if bias is not None else [])
        return [b.node("Conv", ins, strides=stride, pads=pad + pad, dilations=dil, group=int(groups),
                       kernel_shape=list(b.shape(w)[2:]))]
    if k == "batch_norm":
        x, rm, rv = a[0], a[1], a[2]
        w, bb = kw.get("weight"), kw.get("bias")
        C = b.shape(x)[1]
        wv = V(w) if w is not None else b.const([1.0] * C)
        bv = V(bb) if bb is not None else b.const([0.0] * C)
        return [b.node("BatchNormalization", [V(x), wv, bv, V(rm), V(rv)], epsilon=float(kw.get("eps", 1e-5)))]
    if k == "layer_norm":
        x = a[0]
        w = a[1] if len(a) > 1 else None
        bb = a[2] if len(a) > 2 else None
        eps = next((v for v in a[3:] if isinstance(v, float)), 1e-5)
        if not isinstance(w, torch.Tensor):
            return None
        ins = [V(x), V(w)] + ([V(bb)] if isinstance(bb, torch.Tensor) else [])
        return [b.node("LayerNormalization", ins, axis=-1, epsilon=float(eps))]
    if k == "max_pool2d":
        ks = _pair(a[1] if len(a) > 1 else kw["kernel_size"])
        st = _pair(kw.get("stride") or ks)
        pd = _pair(kw.get("padding", 0))
        return [b.node("MaxPool", [V(a[0])], kernel_shape=ks, strides=st, pads=pd + pd,
                       ceil_mode=int(bool(kw.get("ceil_mode", False))))]
    if k == "avg_pool2d":
        ks = _pair(a[1] if len(a) > 1 else kw["kernel_size"])
        st = _pair(kw.get("stride") or ks)
        pd = _pair(kw.get("padding", 0))
        return [b.node("AveragePool", [V(a[0])], kernel_shape=ks, strides=st, pads=pd + pd)]
    if k == "adaptive_avg_pool2d":
        if _pair(a[1] if len(a) > 1 else kw["output_size"]) == [1, 1]:
            return [b.node("GlobalAveragePool", [V(a[0])])]
        return None
    if k == "embedding":
        return [b.node("Gather", [V(a[1]), V(a[0])], axis=0)]
    if k == "cat":
        dim = a[1] if len(a) > 1 else kw.get("dim", 0)
        return [b.node("Concat", [V(t) for t in a[0]], axis=int(dim))]
    return None


def export_program(program, feed_names, fetch, path=None, producer="paddle2_amd"):
    """-> ModelProto bytes for a recorded Program (written to ``path`` when given)."""
    from ..framework.tensor import Tensor

    b = _Builder(program)
    inputs = []
    for n in feed_names:
        sym = program.feeds[n]
        b.names[("v", sym._vid)] = n
        inputs.append(_value_info(n, list(sym.shape), sym.dtype))
    unsupported = []
    for op in program.ops:
        if op.kind not in ("torch", "native"):
            continue
        outs = _convert(b, op)
        if outs is None:
            unsupported.append(op.name)
            continue
        res = [o for o in op.outs if o is not None]
        for vid, name in zip(res, outs):
            b.names[("v", vid)] = name
    if unsupported:
        raise NotImplementedError(f"onnx export: no ONNX mapping for ops {sorted(set(unsupported))}")
    outputs = []
    for i, f in enumerate(fetch):
        t = f._t if isinstance(f, Tensor) else f
        nm = b.names[("v", t._vid)]
        out_name = f"output_{i}"
        b.node("Identity", [nm], [out_name])
        outputs.append(_value_info(out_name, list(t.shape), t.dtype))
    model = {"ir_version": 8, "producer_name": producer, "producer_version": "3",
             "opset_import": [{"domain": "", "version": OPSET}],
             "graph": {"node": b.nodes, "name": "main", "initializer": b.inits, "input": inputs, "output": outputs}}
    data = P.encode(model, "onnx.ModelProto")
    if path:
        d = os.path.dirname(path)
        if d:
            os.makedirs(d, exist_ok=True)
        with open(path, "wb") as fh:
            fh.write(data)
    return data


def load_model_dict(path_or_bytes):
    data = path_or_bytes if isinstance(path_or_bytes, (bytes, bytearray)) else open(path_or_bytes, "rb").read()
    return P.decode(data, "onnx.ModelProto")


def _arr(t):
    return np.frombuffer(t["raw_data"], dtype=_NP[t["data_type"]]).reshape(t.get("dims") or []).copy()


def run_reference(model, feeds):
    """Evaluate a decoded ModelProto with numpy (the op subset the exporter emits)."""
    from scipy.special import erf

    g = model["graph"]
    env = {t["name"]: _arr(t) for t in g["initializer"]}
    env.update({k: np.asarray(v) for k, v in feeds.items()})
    for n in g["node"]:
        at = {x["name"]: x for x in n["attribute"]}
        geti = lambda nm, d=None: at[nm].get("i", d) if nm in at else d  # noqa: E731
        getis = lambda nm, d=None: list(at[nm]["ints"]) if nm in at else d  # noqa: E731
        x = [env[i] for i in n["input"]]
        op = n["op_type"]
        if op == "Gemm":
            y = x[0] @ x[1] + (x[2] if len(x) > 2 else 0)
        elif op == "MatMul":
            y = x[0] @ x[1]
        elif op in ("Add", "Sub", "Mul", "Div", "Pow", "Max", "Min"):
            y = {"Add": np.add, "Sub": np.subtract, "Mul": np.multiply, "Div": np.divide, "Pow": np.power,
                 "Max": np.maximum, "Min": np.minimum}[op](x[0], x[1])
        elif op in ("Relu", "Sigmoid", "Tanh", "Exp", "Log", "Neg", "Sqrt", "Abs", "Erf", "Identity", "Reciprocal"):
            f = {"Relu": lambda v: np.maximum(v, 0), "Sigmoid": lambda v: 1 / (1 + np.exp(-v)), "Tanh": np.tanh,
                 "Exp": np.exp, "Log": np.log, "Neg": np.negative, "Sqrt": np.sqrt, "Abs": np.abs, "Erf": erf,
                 "Identity": lambda v: v, "Reciprocal": lambda v: 1 / v}[op]
            y = f(x[0])
        elif op in ("Softmax", "LogSoftmax"):
            ax = geti("axis", -1)
            e = np.exp(x[0] - x[0].max(ax, keepdims=True))
            y = e / e.sum(ax, keepdims=True)
            y = np.log(y) if op == "LogSoftmax" else y
        elif op == "ReduceMean":
            y = x[0].mean(tuple(getis("axes")), keepdims=bool(geti("keepdims", 1)))
        elif op == "ReduceSum":
            y = x[0].sum(tuple(int(v) for v in x[1]), keepdims=bool(geti("keepdims", 1)))
        elif op == "Reshape":
            y = x[0].reshape([int(v) for v in x[1]])
        elif op == "Transpose":
            y = np.transpose(x[0], getis("perm"))
        elif op == "Conv":
            import torch.nn.functional as F

            pads = getis("pads")
            y = F.conv2d(torch.from_numpy(x[0]), torch.from_numpy(x[1]),
                         torch.from_numpy(x[2]) if len(x) > 2 else None, getis("strides"), pads[:2],
                         getis("dilations"), geti("group", 1)).numpy()
        elif op == "BatchNormalization":
            eps = at["epsilon"]["f"]
            sh = [1, -1] + [1] * (x[0].ndim - 2)
            y = (x[0] - x[3].reshape(sh)) / np.sqrt(x[4].reshape(sh) + eps) * x[1].reshape(sh) + x[2].reshape(sh)
        elif op == "LayerNormalization":
            eps = at["epsilon"]["f"]
            m = x[0].mean(-1, keepdims=True)
            v = x[0].var(-1, keepdims=True)
            y = (x[0] - m) / np.sqrt(v + eps) * x[1] + (x[2] if len(x) > 2 else 0)
        elif op in ("MaxPool", "AveragePool"):
            import torch.nn.functional as F

            f = F.max_pool2d if op == "MaxPool" else F.avg_pool2d
            y = f(torch.from_numpy(x[0]), getis("kernel_shape"), getis("strides"), getis("pads")[:2]).numpy()
        elif op == "GlobalAveragePool":
            y = x[0].mean((2, 3), keepdims=True)
        elif op == "Gather":
            y = np.take(x[0], x[1].astype(np.int64), axis=geti("axis", 0))
        elif op == "Concat":
            y = np.concatenate(x, geti("axis", 0))
        else:
            raise NotImplementedError(op)
        env[n["output"][0]] = np.asarray(y, dtype=np.float32) if np.asarray(y).dtype == np.float64 else y
    return [env[o["name"]] for o in g["output"]]


def export_layer(layer, path, input_spec):
    """Record ``layer`` for ``input_spec`` and write ``{path}.onnx`` (reference paddle.onnx.export)."""
    from ..jit import StaticFunction, _spec_tensors

    was = getattr(layer, "training", False)
    if hasattr(layer, "eval"):
        layer.eval()
    try:
        fwd = getattr(layer, "_dygraph_forward", None) or layer.forward
        sf = StaticFunction(lambda *a: fwd(*a), input_spec)
        with torch.no_grad():
            prog, feeds, outs, _ = sf._record(_spec_tensors(input_spec))
    finally:
        if was and hasattr(layer, "train"):
            layer.train()
    out_path = path if path.endswith(".onnx") else path + ".onnx"
    export_program(prog, feeds, outs, out_path)
    return out_path
