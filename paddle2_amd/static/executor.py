"""Program executor (reference: python/paddle/base/executor.py ``Executor.run`` over the
StandaloneExecutor / PIR interpreter; ``CompiledProgram`` + ``BuildStrategy``).

``run`` replays a recorded Program on real tensors: feeds bind the data variables, each op calls
its recorded function (torch op or native-kernel entry point) with variable ids resolved, the
``backward`` op runs the autograd engine from the loss, ``optimize`` runs the (fused) optimizer.
With ``BuildStrategy.enable_cuda_graph`` a static-shape Program is captured once per feed
signature in a HIP graph (torch.cuda.CUDAGraph) after a warm-up replay, and later runs copy the
feeds into the graph's static input buffers and replay the whole step as one graph launch.
"""
from __future__ import annotations

import weakref

import numpy as np
import torch
from torch.utils import _pytree as pytree

from ..framework.tensor import Tensor
from .graph import Program, SymTensor, VarRef, default_main_program


class Scope:
    def __init__(self):
        self.vars = {}

    def var(self, name):
        return self.vars.setdefault(name, None)

    def find_var(self, name):
        return self.vars.get(name)


_global_scope = Scope()


def global_scope():
    return _global_scope


class BuildStrategy:
    def __init__(self):
        self.enable_cuda_graph = False
        self.fuse_all_optimizer_ops = True
        self.fuse_elewise_add_act_ops = False
        self.enable_inplace = True
        self.memory_optimize = False
        self.build_cinn_pass = False


class ExecutionStrategy:
    def __init__(self):
        self.num_threads = 1
        self.num_iteration_per_drop_scope = 1


class CompiledProgram:
    def __init__(self, program_or_graph, build_strategy=None, exec_strategy=None):
        self._program = program_or_graph
        self._build_strategy = build_strategy or BuildStrategy()
        self._exec_strategy = exec_strategy or ExecutionStrategy()

    def with_data_parallel(self, *a, **k):
        return self


def _feed_tensor(v, sym, device):
    if isinstance(v, Tensor):
        t = v._t
    elif isinstance(v, torch.Tensor):
        t = v
    else:
        t = torch.as_tensor(np.asarray(v))
    if sym is not None and t.dtype != sym.dtype and not (t.dtype == torch.float64 and sym.dtype == torch.float32
                                                         and False):
        t = t.to(sym.dtype)
    return t.to(device)


class _GraphState:
    def __init__(self):
        self.graph = None
        self.static_in = None
        self.static_out = None


class Executor:
    _num_threads = 1   # host worker threads of the async interpreter (ExecutionStrategy.num_threads)

    def __init__(self, place=None):
        from ..framework.place import _parse_device, current_torch_device

        self._device = _parse_device(place) if place is not None else current_torch_device()
        self._graphs = {}
        self._pruned = {}

    def close(self):
        self._graphs.clear()

    # ---------------------------------------------------------------- core replay
    def _run_op(self, op, env, res):
        """Run one recorded instruction over ``env`` (outputs bound in place)."""
        if op.kind in ("torch", "native"):
            out = op.fn(*pytree.tree_map(res, op.args), **pytree.tree_map(res, op.kwargs))
            for vid, val in zip(op.outs, pytree.tree_leaves(out)):
                if vid is not None:
                    env[vid] = val
        elif op.kind == "backward":
            env[op.attrs["loss"]].backward()
        elif op.kind == "grad":
            tgts = [env[v] for v in op.attrs["targets"]]
            ins = [env[v] if isinstance(v, int) else v for v in op.attrs["inputs"]]
            gs = torch.autograd.grad(tgts, ins, allow_unused=True, retain_graph=True)
            for vid, g in zip(op.attrs["outs"], gs):
                env[vid] = g if g is not None else torch.zeros_like(ins[0])
        elif op.kind == "param_grad":
            p = op.attrs["param"]
            g = p._t.grad
            env[op.attrs["out"]] = g if g is not None else torch.zeros_like(p._t)
        elif op.kind == "optimize":
            opt = op.attrs["optimizer"]
            with torch.no_grad():
                opt.step()
            opt.clear_grad(set_to_zero=False)
        elif op.kind == "call":
            # a host instruction a pass inserted (fused gradient all-reduce, gradient merge, sharded step, ...)
            op.attrs["fn"](env)

    def _replay(self, program, env, grad=None, keep=None):
        """Run ``program`` over ``env`` (vid -> tensor) through its interpreter plan (csrc/runtime/interpreter.cpp).

        With ``keep`` (the fetch targets) values are dropped after their last reader.  Device programs issue the
        instructions in the plan's order (kernels are asynchronous on their streams; instructions the stream
        analyzer put on the comm / copy streams run there, and only cross-stream dependency edges get events).
        Host programs with ``ExecutionStrategy.num_threads`` > 1 run on the dependency-counting ready queue: N
        worker threads execute independent instructions concurrently (reference pir_interpreter.cc async work
        queue / RunNextInstructions)."""
        needs_grad = any(o.kind in ("backward", "grad") for o in program.ops) or bool(grad)
        plan = _plan(program, keep if keep is not None else _ALL)
        gc = keep is not None

        def res(x):
            if isinstance(x, VarRef):
                if x.vid not in env:
                    raise RuntimeError(f"variable %{x.vid} has no value (missing feed?)")
                return env[x.vid]
            return x

        on_gpu = torch.cuda.is_available() and self._device.type == "cuda"
        if not on_gpu and self._num_threads > 1 and plan.n > 1:
            return self._replay_async(program, env, plan, needs_grad, gc, res)
        streams = plan.multi_stream and on_gpu
        if streams:
            from ..device.context import get_context

            gctx = get_context(self._device)
            side = {"comm": gctx.comm_stream, "h2d": gctx.h2d_stream, "d2h": gctx.d2h_stream}
            compute = torch.cuda.current_stream(self._device)
            done_ev = {}   # instruction -> event recorded right after it (only producers of cross-stream edges)
        ctx = torch.enable_grad() if needs_grad else torch.no_grad()
        with ctx:
            for i in plan.order:
                op = program.ops[i]
                if streams and (plan.stream_of[i] != "compute" or plan.waits[i]):
                    st = side[plan.stream_of[i]]() if plan.stream_of[i] != "compute" else compute
                    for pi in plan.waits[i]:
                        st.wait_event(done_ev[pi])
                    if st is not compute:
                        for v in plan.reads[i]:
                            if v in env and isinstance(env[v], torch.Tensor) and env[v].is_cuda:
                                env[v].record_stream(st)   # allocator: the side stream still reads it
                    with torch.cuda.stream(st):
                        self._run_op(op, env, res)
                else:
                    self._run_op(op, env, res)
                if streams and plan.record[i]:
                    e = torch.cuda.Event()
                    e.record(side[plan.stream_of[i]]() if plan.stream_of[i] != "compute" else compute)
                    done_ev[i] = e
                if gc:
                    for v in plan.free_after[i]:
                        env.pop(v, None)
        if streams:
            # values produced on a side stream and fetched / left in env: the caller reads them on compute
            for i, e in done_ev.items():
                if plan.stream_of[i] != "compute":
                    compute.wait_event(e)
        return env

    def _replay_async(self, program, env, plan, needs_grad, gc, res):
        import threading

        q = plan.queue()
        q.start()
        errors = []

        def worker():
            with (torch.enable_grad() if needs_grad else torch.no_grad()):  # grad mode is thread-local
                while True:
                    i = q.pop(-1.0)
                    if i < 0:
                        return
                    try:
                        self._run_op(program.ops[i], env, res)
                    except BaseException as e:  # noqa: BLE001 - re-raised on the calling thread
                        errors.append(e)
                        q.fail()
                        return
                    dead = q.done(i)
                    if gc:
                        for v in dead:
                            env.pop(v, None)

        ts = [threading.Thread(target=worker, daemon=True) for _ in range(min(self._num_threads, plan.n))]
        for t in ts:
            t.start()
        for t in ts:
            t.join()
        if errors:
            raise errors[0]
        return env

    def run(self, program=None, feed=None, fetch_list=None, feed_var_name="feed", fetch_var_name="fetch", scope=None,
            return_numpy=True, use_program_cache=False, use_prune=False, _grad=None):
        strategy = None
        self._num_threads = 1
        if isinstance(program, CompiledProgram):
            strategy = program._build_strategy
            self._num_threads = max(1, int(program._exec_strategy.num_threads))
            program = program._program
        program = program or default_main_program()
        from .pdmodel import PdProgram

        if isinstance(program, PdProgram):  # a reference-format model loaded by load_inference_model
            feed = feed or {}
            xs = [_feed_tensor(feed[n], None, self._device) for n in program.feed_names]
            outs = program.run(xs)
            return [o.detach().cpu().numpy() if return_numpy else Tensor._wrap(o) for o in outs]
        if not isinstance(program, Program):
            raise TypeError("Executor.run expects a static Program")
        if getattr(program, "_pipeline_opt", None):
            # minimized by incubate.optimizer.PipelineOptimizer: this rank's pipeline stage over micro-batches
            from ..incubate.optimizer import _run_pipeline

            return _run_pipeline(self, program, feed, fetch_list, return_numpy)
        feed = feed or {}
        fetch_list = fetch_list or []
        if not program.ops and not fetch_list:
            return []  # startup program: parameters are initialised at creation
        fetch_ids = [self._fetch_id(program, f) for f in fetch_list]
        env = {}
        for name, v in feed.items():
            sym = program.feeds.get(name)
            if sym is None:
                raise KeyError(f"feed '{name}' is not a data variable of this program")
            env[sym._vid] = _feed_tensor(v, sym, self._device)
        program = self._executable(program, fetch_ids)
        if strategy is not None and strategy.enable_cuda_graph and self._device.type == "cuda":
            outs = self._run_graph(program, env, fetch_ids)
        else:
            env = self._replay(program, env, _grad, keep=set(fetch_ids))
            outs = [env[i] for i in fetch_ids]
        if return_numpy:
            return [o.detach().float().cpu().numpy() if o.dtype == torch.bfloat16 else o.detach().cpu().numpy()
                    for o in outs]
        return [Tensor._wrap(o if _grad else o.detach()) for o in outs]

    def _executable(self, program, fetch_ids):
        """What runs: the Program translated to PIR, optimised by the pass pipeline (DCE against the fetch targets
        and the side effects, CSE, fused_gemm_epilogue) and lowered back to instructions (pir/lowering.py; reference
        pir_interpreter.cc runs the PIR program after the passes).  FLAGS_enable_pir_in_executor=0 runs the
        recorded instructions as they are (inference programs still pruned to the fetch targets)."""
        from ..framework import flags

        key = (id(program), len(program.ops), tuple(fetch_ids))
        hit = self._pruned.get(key)
        if hit is not None:
            return hit[0]
        train = any(o.kind in ("backward", "grad", "optimize", "param_grad") for o in program.ops)
        if str(flags.flag("FLAGS_enable_pir_in_executor", True)).lower() not in ("0", "false"):
            from ..pir import lowering

            exe_prog, pir_prog, stats = lowering.optimize(program, fetch_ids)
            self._pruned[key] = (exe_prog, program)   # the source program stays alive while its key is cached
            self.last_pir = pir_prog
            self.last_pass_stats = stats
            return exe_prog
        if train:
            return program
        from .io import _prune

        pruned = Program()
        pruned.ops = _prune(program, fetch_ids)
        pruned.feeds, pruned.vars = program.feeds, program.vars
        self._pruned[key] = (pruned, program)
        return pruned

    @staticmethod
    def _fetch_id(program, f):
        if isinstance(f, Tensor):
            f = f._t
        if isinstance(f, SymTensor):
            return f._vid
        if isinstance(f, str):
            for v in program.vars.values():
                if v._name == f:
                    return v._vid
            if f in program.feeds:
                return program.feeds[f]._vid
        raise KeyError(f"cannot fetch {f!r}")

    def _run_graph(self, program, env, fetch_ids):
        key = (id(program), tuple((k, tuple(v.shape), v.dtype) for k, v in sorted(env.items())), tuple(fetch_ids))
        st = self._graphs.get(key)
        if st is None:
            st = _GraphState()
            st.static_in = {k: v.clone() for k, v in env.items()}
            from ..device.context import get_context

            s = get_context().capture_stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(2):
                    e2 = self._replay(program, dict(st.static_in))
            torch.cuda.current_stream().wait_stream(s)
            from ..ops import fp8

            fp8.before_capture()   # the warm-up replays' queued fp8 updates must not enter the graph
            st.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(st.graph):
                e3 = self._replay(program, dict(st.static_in))
            st.static_out = [e3[i] for i in fetch_ids]
            self._graphs[key] = st
        for k, v in env.items():
            st.static_in[k].copy_(v)
        st.graph.replay()
        return [o.clone() for o in st.static_out]


# ==================================================================================== execution plan
_STREAM_IDS = {"compute": 0, "comm": 1, "h2d": 2, "d2h": 3}
_ALL = object()   # keep every value (no garbage collection)


class _Plan:
    """Per-(program, fetch set) interpreter plan, built natively (csrc/runtime/interpreter.cpp; reference
    new_executor/interpreter/dependency_builder.cc, stream_analyzer.cc, pir_interpreter.cc:804):

    * a dependency graph over the instructions from their variable reads / writes (RAW, WAR, WAW), with
      backward / optimizer / in-place instructions as barriers (hidden side effects), transitively reduced;
    * ``order`` — the issue order (topological; communication / copy instructions issued as soon as ready);
    * ``stream_of[i]`` — "compute", or the stream class a function declares via ``_pd_stream`` ("comm" for
      collectives, "h2d" / "d2h" for copies); ``waits[i]`` — producers on another stream whose events op i's
      stream waits on; ``record[i]`` — op i records such an event;
    * ``free_after[i]`` — values whose last reader (in issue order) is op i, dropped right after it unless
      fetched; the async queue frees a value when its reader count drains instead.
    """

    def __init__(self, program, keep):
        from .. import _rt

        ops = program.ops
        self.n = len(ops)
        self.reads = [_op_reads(op) for op in ops]
        writes = [_op_writes(op) for op in ops]
        self.stream_of = [((op.attrs.get("stream") or getattr(op.fn, "_pd_stream", None) or "compute")
                           if op.kind in ("torch", "native") else "compute") for op in ops]
        barrier = [int(op.kind not in ("torch", "native") or bool(set(w) & set(r)))
                   for op, r, w in zip(ops, self.reads, writes)]
        keep_ids = sorted({v for r in self.reads for v in r} | {v for w in writes for v in w}) if keep is _ALL \
            else sorted(keep)
        self.native = _rt.get().build_interp_plan(self.reads, writes,
                                                      [_STREAM_IDS.get(c, 0) for c in self.stream_of], barrier,
                                                      keep_ids)
        self.order = list(self.native.order)
        self.waits = self.native.waits
        self.record = self.native.record
        self.free_after = self.native.free_after
        self.multi_stream = any(k != "compute" for k in self.stream_of)

    def queue(self):
        from .. import _rt

        return _rt.get().ReadyQueue(self.native)


def _op_reads(op):
    vids = [x.vid for x in pytree.tree_leaves((op.args, op.kwargs)) if isinstance(x, VarRef)]
    a = op.attrs
    if "loss" in a:
        vids.append(a["loss"])
    for k in ("targets", "inputs"):
        vids.extend(v for v in a.get(k, ()) if isinstance(v, int))
    return vids


def _op_writes(op):
    out = [v for v in op.outs if v is not None]
    a = op.attrs
    if "out" in a:
        out.append(a["out"])
    out.extend(a.get("outs", ()))
    return out


_PLANS = weakref.WeakKeyDictionary()   # program -> {(num ops, fetch set): plan}


def _plan(program, keep):
    from ..framework import flags

    if float(flags.flag("FLAGS_eager_delete_tensor_gb", 0.0)) < 0:
        keep = _ALL   # garbage collection disabled: keep everything
    per = _PLANS.setdefault(program, {})
    key = (len(program.ops), keep if keep is _ALL else frozenset(keep))
    p = per.get(key)
    if p is None:
        p = per[key] = _Plan(program, keep)
    return p
