"""DRR — declarative rewrite rules for PIR, and the greedy pattern-rewrite driver.

Reference: paddle/fluid/pir/drr/ (DrrPatternBase: a SourcePattern of ops over named tensors and attributes, a
ResultPattern built from the same names, constraints, compiled into a RewritePattern) and
paddle/pir/include/pattern_rewrite/ (RewritePatternSet, ApplyPatternsGreedily).  Here a pattern is written as:

    src = drr.SourcePattern()
    mm = src.op("pd_op.matmul", trans_x=False, trans_y=src.attr("ty"))(src.tensor("x"), src.tensor("w"))
    src.op("pd_op.add")(mm, src.tensor("b"))
    res = drr.ResultPattern(src)
    res.op("pd_op.fused_gemm_epilogue", trans_x=False, trans_y=res.attr("ty"),
           activation="identity")(res.tensor("x"), res.tensor("w"), res.tensor("b"))
    pat = drr.Pattern("gemm_bias", src, res, constraint=lambda m: len(m["b"].shape) == 1)

The source graph is matched anchored at its last op, walking operands to their defining ops; a named tensor
binds one Value (the same name must bind the same Value); attribute literals must be equal and ``attr(name)``
captures the op's attribute for the result pattern.  Intermediate source values must have no users outside the
match (the matched ops are erased).  The result ops are inserted before the anchor and the anchor's results are
replaced by the result pattern's outputs.
"""
from __future__ import annotations

from . import Operation


class _Attr:
    def __init__(self, name):
        self.name = name


class _Tensor:
    def __init__(self, pat, name):
        self.pat, self.name = pat, name


class _OpCall:
    def __init__(self, pat, name, attrs):
        self.pat, self.name, self.attrs = pat, name, attrs
        self.inputs = []
        self.outputs = []

    def __call__(self, *inputs, num_results=1):
        self.inputs = list(inputs)
        self.outputs = [_Tensor(self.pat, f"{self.name}#{len(self.pat.ops)}:{i}") for i in range(num_results)]
        for o in self.outputs:
            o.producer = self
        self.pat.ops.append(self)
        return self.outputs[0] if num_results == 1 else tuple(self.outputs)


class _PatternBase:
    def __init__(self):
        self.ops = []
        self._tensors = {}

    def tensor(self, name):
        t = self._tensors.get(name)
        if t is None:
            t = self._tensors[name] = _Tensor(self, name)
            t.producer = None
        return t

    def attr(self, name):
        return _Attr(name)

    def op(self, name, **attrs):
        return _OpCall(self, name, attrs)


class SourcePattern(_PatternBase):
    pass


class ResultPattern(_PatternBase):
    def __init__(self, src=None):
        super().__init__()
        self.src = src


class Pattern:
    """One rewrite rule: ``constraint(match)`` (optional) sees the bound Values / attributes by name;
    ``compute_attrs(match)`` (optional) returns extra computed attributes the result pattern references with
    ``attr(name)``."""

    def __init__(self, name, src, res, constraint=None, compute_attrs=None, benefit=1):
        if not src.ops:
            raise ValueError(f"pattern {name}: empty source pattern")
        self.name, self.src, self.res = name, src, res
        self.constraint, self.compute_attrs, self.benefit = constraint, compute_attrs, benefit
        self.anchor = src.ops[-1]

    # ------------------------------------------------------------------ matching
    def match(self, op):
        binding = {"__ops__": []}
        if not self._match_op(self.anchor, op, binding):
            return None
        matched = binding["__ops__"]
        # intermediates (results of matched ops other than the anchor) must be used only inside the match
        inside = {id(o) for o in matched}
        for o in matched:
            if o is op:
                continue
            for r in o.results():
                if any(id(u) not in inside for u, _ in r.uses):
                    return None
        if self.constraint is not None and not self.constraint(binding):
            return None
        return binding

    def _match_op(self, pop, op, b):
        if op is None or op.name() != pop.name or op.num_operands() != len(pop.inputs):
            return False
        # the pattern names the leading results; trailing ones (e.g. reshape / transpose XShape) must be unused
        if len(pop.outputs) > op.num_results() or any(not r.use_empty() for r in op.results()[len(pop.outputs):]):
            return False
        for k, v in pop.attrs.items():
            actual = op.attrs_.get(k)
            if isinstance(v, _Attr):
                if v.name in b and b[v.name] != actual:
                    return False
                b[v.name] = actual
            elif actual != v and not (actual is None and v is False):
                return False
        for i, t in enumerate(pop.inputs):
            val = op.operand_source(i)
            if t.producer is not None:
                d = val.get_defining_op()
                if any(d is m for m in b["__ops__"]) or not self._match_op(t.producer, d, b):
                    return False
                if t.producer.outputs.index(t) != d.results().index(val):
                    return False
            else:
                if t.name in b and b[t.name] is not val:
                    return False
                b[t.name] = val
        b["__ops__"].append(op)
        return True

    # ------------------------------------------------------------------ rewriting
    def rewrite(self, program, anchor, b):
        block = program.global_block()
        if self.compute_attrs is not None:
            b.update(self.compute_attrs(b))
        env = dict(b)
        last = None
        for rop in self.res.ops:
            operands = []
            for t in rop.inputs:
                v = env.get(t.name) if t.producer is None else env[id(t)]
                if v is None:
                    raise KeyError(f"pattern {self.name}: result tensor {t.name!r} is not bound by the source")
                operands.append(v)
            attrs = {k: (b[v.name] if isinstance(v, _Attr) else v) for k, v in rop.attrs.items()}
            if len(rop.outputs) == 1 and rop is self.res.ops[-1]:
                rtypes = [(r.shape, r.dtype) for r in anchor.results()][:1]
            else:
                rtypes = [(operands[0].shape, operands[0].dtype)] * len(rop.outputs)
            new = Operation(rop.name, operands, rtypes, attrs)
            block.insert_before(anchor, new)
            for t, r in zip(rop.outputs, new.results()):
                env[id(t)] = r
            last = new
        # a result pattern that is just a source tensor (e.g. x = transpose(transpose(x)))
        outs = [env[id(t)] for t in self.res.ops[-1].outputs] if self.res.ops else [b[self.res._alias]]
        for r, new_r in zip(anchor.results(), outs):
            r.replace_all_uses_with(new_r)
        for o in reversed(b["__ops__"]):
            if o.block is block:
                block.remove_op(o)
        return last


class AliasResult(ResultPattern):
    """Result pattern that forwards a bound source tensor (cancelling rewrites)."""

    def __init__(self, src, name):
        super().__init__(src)
        self._alias = name


class RewritePatternSet:
    def __init__(self, patterns=()):
        self.patterns = sorted(patterns, key=lambda p: -p.benefit)

    def add(self, p):
        self.patterns.append(p)
        self.patterns.sort(key=lambda q: -q.benefit)


def apply_patterns_greedily(program, patterns, max_iterations=10):
    """Rewrite until no pattern matches (or ``max_iterations`` sweeps); returns {pattern name: rewrites}."""
    if not isinstance(patterns, RewritePatternSet):
        patterns = RewritePatternSet(patterns)
    stats = {p.name: 0 for p in patterns.patterns}
    for _ in range(max_iterations):
        changed = False
        # bottom-up: an op is offered to the patterns before its producers, so the largest match anchored at a
        # consumer (GEMM + bias + activation at the activation) wins over a smaller one anchored at a producer
        for op in reversed(list(program.global_block().ops)):
            if op.block is None or op not in program.global_block().ops:
                continue
            for p in patterns.patterns:
                m = p.match(op)
                if m is not None:
                    p.rewrite(program, op, m)
                    stats[p.name] += 1
                    changed = True
                    break
        if not changed:
            break
    return stats


# ============================================================================================ built-in rules
def _gemm_epilogue_patterns():
    out = []
    for act_op, act in ((None, "identity"), ("pd_op.relu", "relu"), ("pd_op.gelu", "gelu")):
        src = SourcePattern()
        mm = src.op("pd_op.matmul", trans_x=False, trans_y=src.attr("ty"))(src.tensor("x"), src.tensor("w"))
        y = src.op("pd_op.add")(mm, src.tensor("b"))
        if act_op:
            src.op(act_op, **({"approximate": src.attr("approx")} if act_op == "pd_op.gelu" else {}))(y)
        res = ResultPattern(src)
        res.op("pd_op.fused_gemm_epilogue", trans_x=False, trans_y=res.attr("ty"),
               activation=res.attr("act"))(res.tensor("x"), res.tensor("w"), res.tensor("b"))

        def constraint(m):
            b, w = m["b"], m["w"]
            return b.shape is not None and len(b.shape) == 1 and w.shape is not None and len(w.shape) == 2

        def attrs(m, act=act):
            a = act
            if act == "gelu" and m.get("approx"):
                a = "gelu_tanh"
            return {"act": a, "ty": bool(m.get("ty") or False)}

        out.append(Pattern(f"fused_gemm_epilogue_{act}", src, res, constraint, attrs, benefit=2 if act_op else 1))
    return out


def _cancel_patterns():
    # transpose(transpose(x, p), q) with q o p = identity  ->  x
    src = SourcePattern()
    t1 = src.op("pd_op.transpose", axis=src.attr("p"))(src.tensor("x"))
    src.op("pd_op.transpose", axis=src.attr("q"))(t1)

    def inverse(m):
        p, q = m.get("p"), m.get("q")
        return p is not None and q is not None and len(p) == len(q) and [p[i] for i in q] == list(range(len(p)))

    cancel_t = Pattern("cancel_transpose_pair", src, AliasResult(src, "x"), inverse, benefit=3)
    # scale(scale(x, a, b), c, d) (bias after scale) -> scale(x, a*c, b*c + d)
    src2 = SourcePattern()
    s1 = src2.op("pd_op.scale", scale=src2.attr("a"), bias=src2.attr("b"), bias_after_scale=True)(src2.tensor("x"))
    src2.op("pd_op.scale", scale=src2.attr("c"), bias=src2.attr("d"), bias_after_scale=True)(s1)
    res2 = ResultPattern(src2)
    res2.op("pd_op.scale", scale=res2.attr("sc"), bias=res2.attr("bs"), bias_after_scale=True)(res2.tensor("x"))
    fold_scale = Pattern("fold_scale_pair", src2, res2,
                         compute_attrs=lambda m: {"sc": float(m["a"]) * float(m["c"]),
                                                  "bs": float(m["b"]) * float(m["c"]) + float(m["d"])}, benefit=3)
    return [cancel_t, fold_scale]


def default_patterns():
    return RewritePatternSet(_gemm_epilogue_patterns() + _cancel_patterns())
