"""PIR passes (reference: paddle/pir/transforms/ — dead_code_elimination_pass, common_subexpression_elimination,
constant_folding_pass; paddle/fluid/pir/transforms/gpu/fused_gemm_epilogue_pass.cc) and a PassManager.

Each pass rewrites a ``pir.Program`` in place and returns the number of rewrites it made."""
from __future__ import annotations

from . import Operation

_SIDE_EFFECT = {"pd_op.fetch", "pd_op.data", "builtin.parameter"}
_IMPURE = {"pd_op.dropout", "pd_op.uniform", "pd_op.gaussian", "pd_op.randint"}
_FOLDABLE = {"pd_op.transpose", "pd_op.reshape", "pd_op.scale", "pd_op.flatten", "pd_op.cast", "pd_op.add",
             "pd_op.multiply", "pd_op.subtract", "pd_op.divide", "pd_op.exp", "pd_op.sqrt", "pd_op.concat"}


def dead_code_elimination_pass(program):
    removed = 0
    changed = True
    while changed:
        changed = False
        for op in list(reversed(program.block.ops)):
            if op.name() in _SIDE_EFFECT and op.name() != "builtin.parameter":
                continue
            if all(r.use_empty() for r in op.results()):
                program.block.remove_op(op)
                if op.name() == "builtin.parameter":
                    program.params.pop(op.result(0).id, None)
                removed += 1
                changed = True
    return removed


def _attr_key(attrs):
    def freeze(v):
        if isinstance(v, (list, tuple)):
            return tuple(freeze(x) for x in v)
        if isinstance(v, dict):
            return tuple(sorted((k, freeze(x)) for k, x in v.items()))
        return v

    return freeze(attrs)


def common_subexpression_elimination_pass(program):
    seen, n = {}, 0
    for op in list(program.block.ops):
        if op.name() in _SIDE_EFFECT or op.name() in _IMPURE:
            continue
        key = (op.name(), tuple(v.id for v in op.operands()), _attr_key(op.attrs()))
        prev = seen.get(key)
        if prev is None:
            seen[key] = op
            continue
        for a, b in zip(op.results(), prev.results()):
            a.replace_all_uses_with(b)
        program.block.remove_op(op)
        n += 1
    return n


def constant_folding_pass(program):
    """Evaluate pure ops whose operands are all parameters/constants once and store the result as a new
    ``builtin.parameter`` (inference programs: e.g. a transposed or rescaled weight)."""
    from . import Program, run

    n = 0
    for op in list(program.block.ops):
        if op.name() not in _FOLDABLE:
            continue
        srcs = [v.get_defining_op() for v in op.operands()]
        if not srcs or not all(s is not None and s.name() == "builtin.parameter" for s in srcs):
            continue
        sub = Program()
        vals = []
        for v in op.operands():
            p = sub.block.append(Operation("builtin.parameter", [], [(v.shape, v.dtype)]))
            sub.params[p.result(0).id] = program.params[v.id]
            vals.append(p.result(0))
        clone = sub.block.append(Operation(op.name(), vals, [(r.shape, r.dtype) for r in op.results()], op.attrs()))
        for i, r in enumerate(clone.results()):
            sub.block.append(Operation("pd_op.fetch", [r], [(r.shape, r.dtype)], {"col": i}))
        res = run(sub, [])
        for i, r in enumerate(op.results()):
            t = res[i].detach()
            p = Operation("builtin.parameter", [], [(list(t.shape), t.dtype)],
                          {"parameter_name": f"constant_folding@_{op.result(i).id}"})
            program.block.insert_before(program.block.ops[0], p)
            program.params[p.result(0).id] = t
            r.replace_all_uses_with(p.result(0))
        program.block.remove_op(op)
        n += 1
    dead_code_elimination_pass(program)
    return n


def _single_use(v):
    return len(v.uses) == 1


def fused_gemm_epilogue_pass(program):
    """matmul(x, W) -> add(., b [1-D]) [-> relu | gelu]  =>  pd_op.fused_gemm_epilogue(x, W, b){activation}:
    one GEMM node + one fused bias-activation kernel instead of three passes over the output."""
    n = 0
    for op in list(program.block.ops):
        if op.name() != "pd_op.matmul" or op.attrs().get("trans_x", False):
            continue
        out = op.result(0)
        if not _single_use(out):
            continue
        add, _ = out.uses[0]
        if add.name() != "pd_op.add" or add.operand_source(0) is not out:
            continue
        bias = add.operand_source(1)
        if bias.shape is None or len(bias.shape) != 1:
            continue
        w = op.operand_source(1)
        if w.shape is None or len(w.shape) != 2:
            continue
        last, act = add, "identity"
        res = add.result(0)
        if _single_use(res):
            nxt, _ = res.uses[0]
            if nxt.name() in ("pd_op.relu", "pd_op.gelu"):
                act = "relu" if nxt.name() == "pd_op.relu" else (
                    "gelu_tanh" if nxt.attrs().get("approximate") else "gelu")
                last = nxt
        fused = Operation("pd_op.fused_gemm_epilogue", [op.operand_source(0), w, bias],
                          [(last.result(0).shape, last.result(0).dtype)],
                          {"trans_x": False, "trans_y": bool(op.attrs().get("trans_y", False)), "activation": act})
        program.block.insert_before(op, fused)
        last.result(0).replace_all_uses_with(fused.result(0))
        for o in ([last] if last is not add else []) + [add, op]:
            program.block.remove_op(o)
        n += 1
    return n


def drr_rewrite_pass(program):
    """The built-in declarative rules (pir/drr.py: GEMM + bias (+ relu / gelu) -> fused_gemm_epilogue, inverse
    transpose pairs cancelled, scale chains folded), applied greedily."""
    from . import drr

    return sum(drr.apply_patterns_greedily(program, drr.default_patterns()).values())


_PASSES = {"drr_rewrite_pass": drr_rewrite_pass,
           "dead_code_elimination_pass": dead_code_elimination_pass,
           "common_subexpression_elimination_pass": common_subexpression_elimination_pass,
           "constant_folding_pass": constant_folding_pass,
           "fused_gemm_epilogue_pass": fused_gemm_epilogue_pass}


class PassManager:
    def __init__(self, passes=None, opt_level=2):
        self.passes = list(passes or [])

    def add_pass(self, name, attrs=None):
        if name not in _PASSES:
            raise ValueError(f"unknown pass {name!r}; available: {sorted(_PASSES)}")
        self.passes.append(name)

    def run(self, program):
        stats = {}
        for p in self.passes:
            stats[p] = _PASSES[p](program)
        return stats


def apply(program, names):
    pm = PassManager()
    for n in names:
        pm.add_pass(n)
    return pm.run(program)
