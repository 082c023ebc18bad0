"""PIR dialects: operation definitions (traits, operand / result arity, attribute schema, verifier, meta
inference) and the program verifier.

Reference: paddle/pir/include/core/ir_context.h + dialect.h (an IrContext owning registered dialects, each
registering its ops' OpInfo), op_info / op_trait / interface (traits such as SideEffect / Pure / Inplace,
VerifySig / InferMetaInterface), paddle/fluid/pir/dialect/operator/ir/op_dialect.cc (the pd_op dialect) and
paddle/pir/src/core/verify.cc (operand dominance and use-list checks).  Here an ``OpInfo`` is a small record;
the pd_op dialect registers the ops the translator (``pir.translate_to_pir``) and the rewrite patterns produce,
and ``verify(program)`` checks the whole SSA program: every op registered (unless the dialect allows unknown
ops), arity, attribute types, operands defined before use in the block, and use lists consistent both ways.
"""
from __future__ import annotations

from dataclasses import dataclass, field

# traits
PURE = "Pure"                 # no side effects: DCE / CSE may remove or merge it
SIDE_EFFECT = "SideEffect"    # never removed (feeds, fetches, random ops)
COMMUTATIVE = "Commutative"   # operands 0 and 1 may swap (CSE canonicalisation)
INPLACE = "Inplace"           # result 0 aliases operand 0
ELEMENTWISE = "Elementwise"   # result shape = broadcast of operand shapes


class VerifyError(Exception):
    pass


@dataclass
class OpInfo:
    name: str
    operands: tuple = (0, None)          # (min, max) operand count; max None = unbounded
    results: tuple = (1, 1)
    attrs: dict = field(default_factory=dict)   # attribute name -> python type (or tuple of types)
    traits: frozenset = frozenset()
    verify: object = None                # optional fn(op) raising VerifyError
    infer_meta: object = None            # optional fn(operand values, attrs) -> [(shape, dtype)]

    def has_trait(self, t):
        return t in self.traits


class Dialect:
    def __init__(self, name, allow_unknown_ops=False):
        self.name = name
        self.allow_unknown_ops = allow_unknown_ops
        self.ops = {}

    def register_op(self, info):
        if not info.name.startswith(self.name + "."):
            raise ValueError(f"op {info.name} does not belong to dialect {self.name}")
        self.ops[info.name] = info
        return info


class IrContext:
    """Process-wide registry of dialects (reference pir::IrContext::Instance())."""

    _inst = None

    def __init__(self):
        self.dialects = {}

    @classmethod
    def instance(cls):
        if cls._inst is None:
            cls._inst = IrContext()
            _register_builtin(cls._inst)
        return cls._inst

    def register_dialect(self, d):
        self.dialects[d.name] = d
        return d

    def get_dialect(self, name):
        return self.dialects.get(name)

    def op_info(self, op_name):
        d = self.dialects.get(op_name.split(".", 1)[0])
        return None if d is None else d.ops.get(op_name)


def op_info(op_name):
    return IrContext.instance().op_info(op_name)


def has_trait(op, trait):
    info = op_info(op.name())
    return info is not None and info.has_trait(trait)


# ============================================================================================ verification
def _check_attrs(op, info):
    for k, ty in info.attrs.items():
        if k in op.attrs_ and op.attrs_[k] is not None and not isinstance(op.attrs_[k], ty):
            raise VerifyError(f"{op.name()}: attribute {k!r} should be {ty}, got {type(op.attrs_[k]).__name__}")


def verify(program):
    """Raise VerifyError on the first malformed op; return the number of ops checked."""
    ctx = IrContext.instance()
    defined = set()
    ops = program.global_block().ops
    for idx, op in enumerate(ops):
        dname = op.name().split(".", 1)[0]
        d = ctx.get_dialect(dname)
        if d is None:
            raise VerifyError(f"op #{idx} {op.name()}: dialect {dname!r} is not registered")
        info = d.ops.get(op.name())
        if info is None and not d.allow_unknown_ops:
            raise VerifyError(f"op #{idx} {op.name()}: not registered in dialect {dname!r}")
        for i, v in enumerate(op.operands()):
            if v.id not in defined:
                raise VerifyError(f"op #{idx} {op.name()}: operand {i} (%{v.id}) is used before its definition")
            if not any(o is op and j == i for o, j in v.uses):
                raise VerifyError(f"op #{idx} {op.name()}: operand {i} missing from the use list of %{v.id}")
        for r in op.results():
            if r.get_defining_op() is not op:
                raise VerifyError(f"op #{idx} {op.name()}: result %{r.id} points at another defining op")
            for user, j in r.uses:
                if user.block is not op.block or j >= user.num_operands() or user.operand_source(j) is not r:
                    raise VerifyError(f"%{r.id}: stale use by {user.name()} operand {j}")
            defined.add(r.id)
        if info is not None:
            lo, hi = info.operands
            if op.num_operands() < lo or (hi is not None and op.num_operands() > hi):
                raise VerifyError(f"op #{idx} {op.name()}: {op.num_operands()} operands, expected [{lo}, {hi}]")
            rlo, rhi = info.results
            if op.num_results() < rlo or (rhi is not None and op.num_results() > rhi):
                raise VerifyError(f"op #{idx} {op.name()}: {op.num_results()} results, expected [{rlo}, {rhi}]")
            _check_attrs(op, info)
            if info.verify is not None:
                info.verify(op)
    return len(ops)


# ============================================================================================ registrations
def _verify_matmul(op):
    a, b = op.operand_source(0), op.operand_source(1)
    if a.shape and b.shape and len(a.shape) >= 2 and len(b.shape) >= 2:
        ka = a.shape[-1] if not op.attrs_.get("trans_x") else a.shape[-2]
        kb = b.shape[-2] if not op.attrs_.get("trans_y") else b.shape[-1]
        if ka is not None and kb is not None and ka >= 0 and kb >= 0 and ka != kb:
            raise VerifyError(f"pd_op.matmul: reduction sizes differ ({ka} vs {kb})")


def _verify_fge(op):
    w, b = op.operand_source(1), op.operand_source(2)
    if w.shape and b.shape and len(b.shape) == 1:
        n = w.shape[0] if op.attrs_.get("trans_y") else w.shape[-1]
        if n >= 0 and b.shape[0] >= 0 and n != b.shape[0]:
            raise VerifyError("pd_op.fused_gemm_epilogue: bias length differs from the output columns")
    if op.attrs_.get("activation", "identity") not in ("identity", "relu", "gelu", "gelu_tanh", "silu"):
        raise VerifyError(f"pd_op.fused_gemm_epilogue: unknown activation {op.attrs_.get('activation')!r}")


def _register_builtin(ctx):
    builtin = ctx.register_dialect(Dialect("builtin"))
    builtin.register_op(OpInfo("builtin.parameter", (0, 0), (1, 1), {"parameter_name": str},
                               frozenset({SIDE_EFFECT})))
    builtin.register_op(OpInfo("builtin.constant", (0, 0), (1, 1), {}, frozenset({PURE})))
    # pd_op: the Paddle operator dialect.  Ops lowered from the ProgramDesc table that have no entry here still
    # verify (allow_unknown_ops), as in the reference where every op of the yaml set is registered.
    pd = ctx.register_dialect(Dialect("pd_op", allow_unknown_ops=True))
    reg = pd.register_op
    reg(OpInfo("pd_op.data", (0, 0), (1, 1), {"name": str, "col": int}, frozenset({SIDE_EFFECT})))
    reg(OpInfo("pd_op.fetch", (1, 1), (1, 1), {"name": str, "col": int}, frozenset({SIDE_EFFECT})))
    reg(OpInfo("pd_op.matmul", (2, 2), (1, 1), {"trans_x": bool, "trans_y": bool}, frozenset({PURE}),
               verify=_verify_matmul))
    reg(OpInfo("pd_op.fused_gemm_epilogue", (3, 3), (1, 1), {"trans_x": bool, "trans_y": bool, "activation": str},
               frozenset({PURE}), verify=_verify_fge))
    for n in ("add", "multiply"):
        reg(OpInfo(f"pd_op.{n}", (2, 2), (1, 1), {"axis": int}, frozenset({PURE, ELEMENTWISE, COMMUTATIVE})))
    for n in ("subtract", "divide", "maximum", "minimum", "pow"):
        reg(OpInfo(f"pd_op.{n}", (2, 2), (1, 1), {"axis": int}, frozenset({PURE, ELEMENTWISE})))
    for n in ("relu", "gelu", "silu", "sigmoid", "tanh", "exp", "sqrt", "rsqrt", "erf", "abs", "log", "hardswish",
              "swish", "softsign", "leaky_relu", "relu6"):
        reg(OpInfo(f"pd_op.{n}", (1, 1), (1, 1), {}, frozenset({PURE, ELEMENTWISE})))
    reg(OpInfo("pd_op.scale", (1, 2), (1, 1), {"scale": (int, float), "bias": (int, float),
                                               "bias_after_scale": bool}, frozenset({PURE, ELEMENTWISE})))
    reg(OpInfo("pd_op.cast", (1, 1), (1, 1), {}, frozenset({PURE, ELEMENTWISE})))
    for n in ("reshape", "transpose", "flatten", "squeeze", "unsqueeze"):
        reg(OpInfo(f"pd_op.{n}", (1, 2), (1, 2), {}, frozenset({PURE})))
    for n in ("softmax", "log_softmax"):
        reg(OpInfo(f"pd_op.{n}", (1, 1), (1, 1), {"axis": int}, frozenset({PURE})))
    reg(OpInfo("pd_op.layer_norm", (1, 3), (1, 3), {"epsilon": float, "begin_norm_axis": int}, frozenset({PURE})))
    reg(OpInfo("pd_op.rms_norm", (1, 3), (1, 3), {"epsilon": float}, frozenset({PURE})))
    for n in ("sum", "mean", "max", "min"):
        reg(OpInfo(f"pd_op.{n}", (1, 2), (1, 1), {"keepdim": bool}, frozenset({PURE})))
    reg(OpInfo("pd_op.concat", (1, None), (1, 1), {"axis": int}, frozenset({PURE})))
    reg(OpInfo("pd_op.full", (0, 0), (1, 1), {}, frozenset({PURE})))
    reg(OpInfo("pd_op.embedding", (2, 2), (1, 1), {}, frozenset({PURE})))
    for n in ("dropout", "uniform", "gaussian", "randint"):
        reg(OpInfo(f"pd_op.{n}", (0, None), (1, 2), {}, frozenset({SIDE_EFFECT})))
