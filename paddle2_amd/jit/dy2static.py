"""dy2static: AST conversion of tensor-dependent Python control flow (reference:
python/paddle/jit/dy2static/ — IfElseTransformer, LoopTransformer, convert_operators.convert_ifelse /
convert_while_loop).

``convert_function(fn)`` rewrites the function's source so that

    if <test>:            ->   (a, b) = _jst.IfElse(<test>, __true_k, __false_k, (a, b))
        body                   with __true_k / __false_k taking and returning every name either branch assigns
    else:
        orelse

    while <test>:         ->   (a, b) = _jst.While(__cond_k, __body_k, (a, b))
        body                   over the names the loop assigns

and the run-time helpers pick the semantics from the predicate: a Python value (or an eager tensor) keeps
ordinary Python control flow; a symbolic tensor (while ``to_static`` records a Program) becomes
``static.nn.cond`` / ``static.nn.while_loop``, so a data-dependent branch or loop is captured instead of
failing on ``bool(symbolic)``.  Statements the conversion does not model (``return`` / ``break`` / ``continue``
inside the converted block, ``global`` / ``nonlocal``) are left as Python.  Functions without retrievable source
are returned unchanged.
"""
from __future__ import annotations

import ast
import functools
import inspect
import textwrap


class _Undefined:
    def __repr__(self):
        return "<undefined>"


UNDEF = _Undefined()


def get_local(scope, name):
    return scope.get(name, UNDEF)


def _is_sym(x):
    from ..static.nn import _is_sym as s

    return s(x)


def IfElse(pred, true_fn, false_fn, args):
    from ..framework.tensor import Tensor
    from ..static import nn as snn

    if _is_sym(pred):
        return snn.cond(pred, lambda: true_fn(*args), lambda: false_fn(*args))
    if isinstance(pred, Tensor):
        pred = bool(pred._t.reshape(-1)[0]) if pred._t.numel() else False
    return true_fn(*args) if pred else false_fn(*args)


def While(cond_fn, body_fn, args):
    from ..framework.tensor import Tensor
    from ..static import nn as snn

    args = tuple(args)
    first = cond_fn(*args)
    if _is_sym(first) or any(_is_sym(a) for a in args if isinstance(a, Tensor)):
        if not _is_sym(first) and not isinstance(first, Tensor):
            # Python predicate over symbolic state: the trip count is static -> unroll while recording
            while first:
                args = tuple(body_fn(*args))
                first = cond_fn(*args)
            return args
        # names first bound inside the body are loop temporaries, not loop-carried state
        keep = [i for i, a in enumerate(args) if a is not UNDEF]
        if any(not isinstance(args[i], Tensor) for i in keep):
            raise NotImplementedError("dy2static while: loop-carried variables must be Tensors under a tensor "
                                      "predicate")

        def full(a):
            vals = [UNDEF] * len(args)
            for i, v in zip(keep, a):
                vals[i] = v
            return vals

        out = snn.while_loop(lambda *a: cond_fn(*full(a)),
                             lambda *a: tuple(tuple(body_fn(*full(a)))[i] for i in keep),
                             [args[i] for i in keep])
        return tuple(full(out))
    c = first
    while (bool(c._t.reshape(-1)[0]) if isinstance(c, Tensor) else c):
        args = tuple(body_fn(*args))
        c = cond_fn(*args)
    return args


# ================================================================================================ transform
class _Names(ast.NodeVisitor):
    def __init__(self):
        self.stored, self.loaded = [], []
        self.unsupported = False

    def visit_Name(self, node):
        lst = self.stored if isinstance(node.ctx, ast.Store) else self.loaded
        if node.id not in lst and not node.id.startswith("__pd_"):
            lst.append(node.id)

    def visit_FunctionDef(self, node):  # do not descend into nested defs (their locals are not ours)
        if node.name not in self.stored and not node.name.startswith("__pd_"):
            self.stored.append(node.name)

    visit_AsyncFunctionDef = visit_FunctionDef

    def visit_Lambda(self, node):
        pass

    def visit_Return(self, node):
        self.unsupported = True

    def visit_Break(self, node):
        self.unsupported = True

    visit_Continue = visit_Break

    def visit_Global(self, node):
        self.unsupported = True

    visit_Nonlocal = visit_Global


def _names(stmts):
    v = _Names()
    for s in stmts:
        v.visit(s)
    return v


class _Transformer(ast.NodeTransformer):
    def __init__(self):
        self.k = 0

    def _tuple(self, names, ctx):
        return ast.Tuple(elts=[ast.Name(id=n, ctx=ctx()) for n in names], ctx=ctx())

    def _fn(self, name, params, body, ret):
        return ast.FunctionDef(
            name=name,
            args=ast.arguments(posonlyargs=[], args=[ast.arg(arg=p) for p in params], kwonlyargs=[],
                               kw_defaults=[], defaults=[]),
            body=list(body) + [ast.Return(value=ret)], decorator_list=[], returns=None, type_comment=None)

    def _args(self, names):
        # (_jst.get_local(locals(), 'a'), ...): names not yet bound enter as UNDEF
        return ast.Tuple(elts=[ast.Call(func=ast.Attribute(value=ast.Name(id="_jst", ctx=ast.Load()),
                                                           attr="get_local", ctx=ast.Load()),
                                        args=[ast.Call(func=ast.Name(id="locals", ctx=ast.Load()), args=[],
                                                       keywords=[]), ast.Constant(value=n)], keywords=[])
                               for n in names], ctx=ast.Load())

    def visit_If(self, node):
        self.generic_visit(node)
        info = _names(node.body + node.orelse)
        if info.unsupported or not info.stored:
            return node
        names = info.stored
        k = self.k
        self.k += 1
        tname, fname = f"__pd_true_{k}", f"__pd_false_{k}"
        ret = self._tuple(names, ast.Load)
        tdef = self._fn(tname, names, node.body, ret)
        fdef = self._fn(fname, names, node.orelse or [ast.Pass()], self._tuple(names, ast.Load))
        call = ast.Call(func=ast.Attribute(value=ast.Name(id="_jst", ctx=ast.Load()), attr="IfElse", ctx=ast.Load()),
                        args=[node.test, ast.Name(id=tname, ctx=ast.Load()), ast.Name(id=fname, ctx=ast.Load()),
                              self._args(names)], keywords=[])
        assign = ast.Assign(targets=[self._tuple(names, ast.Store)], value=call)
        return [tdef, fdef, assign]

    def visit_While(self, node):
        self.generic_visit(node)
        info = _names(node.body)
        if info.unsupported or node.orelse or not info.stored:
            return node
        names = [n for n in info.stored]
        k = self.k
        self.k += 1
        cname, bname = f"__pd_cond_{k}", f"__pd_body_{k}"
        cdef = self._fn(cname, names, [], node.test)
        bdef = self._fn(bname, names, node.body, self._tuple(names, ast.Load))
        call = ast.Call(func=ast.Attribute(value=ast.Name(id="_jst", ctx=ast.Load()), attr="While", ctx=ast.Load()),
                        args=[ast.Name(id=cname, ctx=ast.Load()), ast.Name(id=bname, ctx=ast.Load()),
                              self._args(names)], keywords=[])
        assign = ast.Assign(targets=[self._tuple(names, ast.Store)], value=call)
        return [cdef, bdef, assign]


@functools.lru_cache(maxsize=None)
def _convert_code(fn):
    try:
        src = textwrap.dedent(inspect.getsource(fn))
    except (OSError, TypeError):
        return None
    tree = ast.parse(src)
    fdef = tree.body[0]
    if not isinstance(fdef, (ast.FunctionDef, ast.AsyncFunctionDef)):
        return None
    fdef.decorator_list = []  # the converted function is the undecorated body
    fdef.args.defaults = []   # defaults are re-attached from the original function object
    fdef.args.kw_defaults = [None] * len(fdef.args.kwonlyargs)
    if "__class__" in fn.__code__.co_freevars and fdef.args.args:
        # zero-argument super() inside a generated branch function would bind that function's first
        # parameter: make it explicit against the original method's instance argument
        me = fdef.args.args[0].arg
        for node in ast.walk(fdef):
            if (isinstance(node, ast.Call) and isinstance(node.func, ast.Name) and node.func.id == "super"
                    and not node.args):
                node.args = [ast.Name(id="__class__", ctx=ast.Load()), ast.Name(id=me, ctx=ast.Load())]
    tr = _Transformer()
    fdef = tr.visit(fdef)
    if tr.k == 0:
        return None
    # wrap in a factory over the original free variables so closures (and the ``__class__`` cell that
    # zero-argument ``super()`` needs) stay real closures
    free = list(fn.__code__.co_freevars)
    factory = ast.FunctionDef(
        name="__pd_factory",
        args=ast.arguments(posonlyargs=[], args=[ast.arg(arg=v) for v in free], kwonlyargs=[], kw_defaults=[],
                           defaults=[]),
        body=[fdef, ast.Return(value=ast.Name(id=fdef.name, ctx=ast.Load()))], decorator_list=[], returns=None,
        type_comment=None)
    mod = ast.Module(body=[factory], type_ignores=[])
    ast.fix_missing_locations(mod)
    return compile(mod, filename=f"<dy2static {fn.__qualname__}>", mode="exec"), free


def convert_function(fn):
    """-> a converted function (or ``fn`` itself when nothing needs converting / no source)."""
    import sys

    if getattr(fn, "__pd_converted__", False):
        return fn
    inner = getattr(fn, "__func__", fn)
    res = _convert_code(inner)
    if res is None:
        return fn
    code, free = res
    glb = inner.__globals__
    if glb.get("_jst") is not sys.modules[__name__]:
        glb = dict(glb)  # keep the module's namespace untouched; a snapshot carries the helper module
        glb["_jst"] = sys.modules[__name__]
    cells = []
    for cell in (inner.__closure__ or ()):
        try:
            cells.append(cell.cell_contents)
        except ValueError:
            cells.append(UNDEF)
    ns = {}
    exec(code, glb, ns)
    new = ns["__pd_factory"](*cells)
    new.__defaults__ = inner.__defaults__
    new.__kwdefaults__ = inner.__kwdefaults__
    new.__pd_converted__ = True
    functools.update_wrapper(new, inner)
    if hasattr(fn, "__self__"):
        return new.__get__(fn.__self__, type(fn.__self__))
    return new
