"""paddle.incubate.optimizer (reference: python/paddle/incubate/optimizer/ — lookahead.py, modelaverage.py,
gradient_merge.py, recompute.py, pipeline.py, lars_momentum.py, distributed_fused_lamb.py, lbfgs.py, functional/).

Meta-optimizers wrap an inner optimizer of ``paddle.optimizer``:

* ``LookAhead`` — k fast steps, then the slow weights move ``alpha`` of the way to the fast ones and the fast
  weights restart from them (Zhang et al. 2019);
* ``ModelAverage`` — running parameter sums over a sliding window (the ``average_accumulates`` kernel's three-sum
  scheme) with ``apply()`` / ``restore()`` to evaluate on the averaged weights;
* ``GradientMergeOptimizer`` — the inner step every ``k_steps`` calls on the summed (or averaged) gradients;
* ``RecomputeOptimizer`` — static graphs: ``minimize`` records the backward with the ``_set_checkpoints``
  segments recomputed (static.append_backward checkpoints), dygraph: a plain step;
* ``PipelineOptimizer`` — static pipeline training: the minimized Program is split by its
  ``device_guard("gpu:<stage>")`` annotations and ``Executor.run`` drives this rank's stage through the 1F1B job
  list of ``num_microbatches`` micro-batches (distributed/passes/pipeline_scheduler_pass.StagePlanExecutor);
* ``LarsMomentumOptimizer`` / ``DistributedFusedLamb`` — LARS momentum and LAMB with their reference names and
  arguments; on several ranks DistributedFusedLamb reduce-scatters the flat gradient, updates its own shard of
  the LAMB state and all-gathers the parameters (ZeRO-1 form of the reference's fused distributed kernel).
"""
from __future__ import annotations

import torch

from ...framework.tensor import Tensor
from ...optimizer import Lamb, Momentum, Optimizer
from ...optimizer.lbfgs import LBFGS  # noqa: F401
from . import functional  # noqa: F401

__all__ = ["LookAhead", "ModelAverage", "GradientMergeOptimizer", "RecomputeOptimizer", "PipelineOptimizer",
           "LarsMomentumOptimizer", "DistributedFusedLamb", "LBFGS", "functional"]


class _Wrapper:
    """Forwarding base of the meta-optimizers: everything not overridden goes to the inner optimizer."""

    def __init__(self, inner):
        self.inner_optimizer = inner

    def __getattr__(self, name):
        if name == "inner_optimizer":
            raise AttributeError(name)
        return getattr(self.inner_optimizer, name)

    def clear_grad(self, set_to_zero=True):
        self.inner_optimizer.clear_grad(set_to_zero)

    clear_gradients = clear_grad

    def state_dict(self):
        return self.inner_optimizer.state_dict()

    def set_state_dict(self, sd):
        self.inner_optimizer.set_state_dict(sd)


class LookAhead(_Wrapper):
    """reference lookahead.py:132 — slow <- slow + alpha (fast - slow) and fast <- slow every k inner steps."""

    def __init__(self, inner_optimizer, alpha=0.5, k=5, name=None):
        if inner_optimizer is None:
            raise ValueError("inner optimizer can not be None")
        if not 0.0 <= alpha <= 1.0:
            raise ValueError("alpha should be in [0, 1]")
        if not (isinstance(k, int) and k > 0):
            raise ValueError("k should be a positive integer")
        super().__init__(inner_optimizer)
        self.alpha, self.k, self._name = float(alpha), int(k), name
        self._slow = {}
        self._count = 0

    @torch.no_grad()
    def step(self):
        params = self.inner_optimizer._parameter_list
        if not self._slow:   # the slow weights start at the weights before the first fast step
            for p in params:
                self._slow[p.name] = p._t.detach().clone()
        self.inner_optimizer.step()
        self._count += 1
        if self._count % self.k == 0:
            for p in params:
                s = self._slow[p.name]
                s.add_(p._t.to(s.dtype) - s, alpha=self.alpha)
                p._t.copy_(s.to(p._t.dtype))

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()
        return None, [(p, Tensor._wrap(p._t.grad)) for p in self.inner_optimizer._parameter_list
                      if p._t.grad is not None]

    def state_dict(self):
        sd = self.inner_optimizer.state_dict()
        for k, v in self._slow.items():
            sd[f"{k}_slow_0"] = Tensor._wrap(v)
        sd["lookahead_step"] = self._count
        return sd

    def set_state_dict(self, sd):
        sd = dict(sd)
        self._count = int(sd.pop("lookahead_step", self._count))
        for k in [k for k in sd if k.endswith("_slow_0")]:
            v = sd.pop(k)
            self._slow[k[:-len("_slow_0")]] = (v._t if isinstance(v, Tensor) else torch.as_tensor(v)).clone()
        self.inner_optimizer.set_state_dict(sd)


class ModelAverage(Optimizer):
    """reference modelaverage.py:191 — per parameter sum_1 / sum_2 / sum_3 and the accumulate counters of the
    ``average_accumulates`` kernel; ``apply()`` swaps in (sum_1 + sum_2 + sum_3) / (num_accumulates +
    old_num_accumulates), ``restore()`` puts the trained weights back."""

    def __init__(self, average_window_rate, parameters=None, min_average_window=10000, max_average_window=10000,
                 name=None):
        super().__init__(0.0, parameters, None, None, name)
        self.average_window = float(average_window_rate)
        self.min_average_window, self.max_average_window = int(min_average_window), int(max_average_window)
        self._backup = {}

    def _state(self, p):
        d = self._accumulators
        if p.name not in d["sum_1"]:
            for k in ("sum_1", "sum_2", "sum_3"):
                d[k][p.name] = torch.zeros_like(p._t, dtype=torch.float32)
            for k in ("num_accumulates", "old_num_accumulates", "num_updates"):
                d[k][p.name] = torch.zeros(1, dtype=torch.int64, device=p._t.device)
        return [d[k][p.name] for k in ("sum_1", "sum_2", "sum_3", "num_accumulates", "old_num_accumulates",
                                       "num_updates")]

    @torch.no_grad()
    def step(self):
        from ...ops.extra_ops import average_accumulates_

        for p in self._parameter_list:
            if getattr(p, "trainable", True) is False:
                continue
            average_accumulates_(p._t, *self._state(p), average_window=self.average_window,
                                 max_average_window=self.max_average_window,
                                 min_average_window=self.min_average_window)

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        self.step()
        return None, []

    def _apply(self, pg):   # step() does not go through the gradient path
        pass

    @torch.no_grad()
    def _swap_in(self):
        for p in self._parameter_list:
            s1, s2, s3, na, ona, _ = self._state(p)
            n = int(na.item()) + int(ona.item())
            if n == 0:
                continue
            self._backup[p.name] = p._t.detach().clone()
            p._t.copy_(((s1 + s2 + s3) / n).to(p._t.dtype))

    def apply(self, executor=None, need_restore=True):
        """Context manager: inside, the parameters hold their window averages (restored on exit when
        ``need_restore``)."""
        outer = self

        class _Ctx:
            def __enter__(self):
                outer._swap_in()
                return outer

            def __exit__(self, *exc):
                if need_restore:
                    outer.restore()
                return False

        return _Ctx()

    @torch.no_grad()
    def restore(self, executor=None):
        for p in self._parameter_list:
            b = self._backup.pop(p.name, None)
            if b is not None:
                p._t.copy_(b)


class GradientMergeOptimizer(_Wrapper):
    """reference gradient_merge.py — the inner optimizer steps every ``k_steps`` calls on the gradients
    accumulated since (averaged when ``avg``); the calls in between leave the accumulated gradients in place."""

    def __init__(self, inner_optimizer, k_steps=1, avg=True):
        if k_steps < 1:
            raise ValueError("k_steps must be >= 1")
        super().__init__(inner_optimizer)
        self.k_steps, self.avg = int(k_steps), bool(avg)
        self._calls = 0

    @torch.no_grad()
    def step(self):
        self._calls += 1
        if self._calls % self.k_steps:
            return False
        if self.avg and self.k_steps > 1:
            for p in self.inner_optimizer._parameter_list:
                if p._t.grad is not None:
                    p._t.grad.div_(self.k_steps)
        self.inner_optimizer.step()
        return True

    def minimize(self, loss, startup_program=None, parameters=None, no_grad_set=None):
        from ...static.graph import SymTensor

        if isinstance(getattr(loss, "_t", None), SymTensor):
            from ...distributed.auto_parallel.static.passes import gradient_merge_pass

            out = self.inner_optimizer.minimize(loss, startup_program, parameters, no_grad_set)

            class _P:
                program = loss._t._program

            gradient_merge_pass(_P, self.k_steps, self.avg)
            return out
        stepped = self.step()
        if stepped:
            self.inner_optimizer.clear_grad(set_to_zero=False)
        return None, []

    def clear_grad(self, set_to_zero=True):
        """Gradients are kept across the merged calls: cleared only right after the inner step."""
        if self._calls % self.k_steps == 0:
            self.inner_optimizer.clear_grad(set_to_zero)


class RecomputeOptimizer(_Wrapper):
    """reference recompute.py — ``_set_checkpoints`` names the tensors kept from the forward; a static
    ``minimize`` records the backward with the segments between them recomputed."""

    def __init__(self, optimizer):
        super().__init__(optimizer)
        self._checkpoints = None

    def _set_checkpoints(self, checkpoints):
        if not isinstance(checkpoints, (list, tuple)):
            raise TypeError("checkpoints should be a list of Tensors")
        self._checkpoints = list(checkpoints)

    def backward(self, loss, startup_program=None, parameter_list=None, no_grad_set=None, callbacks=None):
        from ... import static as _static
        from ...static.graph import SymTensor

        if isinstance(getattr(loss, "_t", None), SymTensor):
            return _static.append_backward(loss, parameter_list, no_grad_set, callbacks,
                                           checkpoints=self._checkpoints)
        loss.backward()
        return [(p, Tensor._wrap(p._t.grad)) for p in self.inner_optimizer._parameter_list if p._t.grad is not None]

    def apply_optimize(self, loss, startup_program, params_grads):
        from ...static.graph import SymTensor

        if isinstance(getattr(loss, "_t", None), SymTensor):
            loss._t._program.append_special("optimize", optimizer=self.inner_optimizer)
            return []
        self.inner_optimizer.step()
        return []

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from ...static.graph import SymTensor

        if isinstance(getattr(loss, "_t", None), SymTensor):
            pg = self.backward(loss, startup_program, parameter_list, no_grad_set)
            self.apply_optimize(loss, startup_program, pg)
            return [], pg
        self.inner_optimizer.step()
        return None, []

    def step(self):
        self.inner_optimizer.step()


class PipelineOptimizer(_Wrapper):
    """reference incubate/optimizer/pipeline.py:94 — static pipeline training.  ``minimize`` records the inner
    optimizer into the Program and marks it for pipelining; ``paddle.static.Executor.run`` then splits the fed
    batch into ``num_microbatches`` along dim 0 and runs this rank's stage (``device_guard("gpu:<stage>")``
    annotations; stage = rank in the pipeline group) through the 1F1B job list (FThenB when the micro-batches do
    not cover the 1F1B warm-up).  ``run`` returns the fetches this stage holds: per-micro-batch scalars averaged,
    others concatenated, values of other stages as None."""

    def __init__(self, optimizer, num_microbatches=1, start_cpu_core_id=0, schedule_mode="1F1B", pp_ranks=None,
                 dp_group=None):
        super().__init__(optimizer)
        if num_microbatches < 1:
            raise ValueError("num_microbatches must be >= 1")
        self._num_microbatches = int(num_microbatches)
        self._start_cpu_core_id = start_cpu_core_id
        self._schedule = schedule_mode
        self._pp_ranks, self._dp_group = pp_ranks, dp_group

    def minimize(self, loss, startup_program=None, parameter_list=None, no_grad_set=None):
        from ...static.graph import SymTensor

        if not isinstance(getattr(loss, "_t", None), SymTensor):
            raise RuntimeError("PipelineOptimizer works on static programs (paddle.enable_static())")
        out = self.inner_optimizer.minimize(loss, startup_program, parameter_list, no_grad_set)
        prog = loss._t._program
        prog._pipeline_opt = {"num_microbatches": self._num_microbatches, "schedule_mode": self._schedule,
                              "pp_ranks": self._pp_ranks, "dp_group": self._dp_group, "runner": None}
        return out


def _run_pipeline(executor, program, feed, fetch_list, return_numpy):
    """Executor.run for a Program minimized by PipelineOptimizer."""
    import numpy as np
    import torch.distributed as tdist

    from ...distributed.passes import StagePlanExecutor, apply_pass

    cfg = program._pipeline_opt
    m = cfg["num_microbatches"]
    runner = cfg["runner"]
    if runner is None:
        pp = cfg["pp_ranks"] or list(range(tdist.get_world_size() if tdist.is_initialized() else 1))
        rank = tdist.get_rank() if tdist.is_initialized() else 0
        stage, degree = pp.index(rank), len(pp)
        mode = cfg["schedule_mode"]
        if mode == "1F1B" and m < degree - stage:
            mode = "FThenB"
        plan = apply_pass(program, mode, m, stage, degree)
        runner = cfg["runner"] = StagePlanExecutor(program, plan, pp, executor, cfg["dp_group"])
    micro = [dict() for _ in range(m)]
    for name, v in (feed or {}).items():
        t = v._t if isinstance(v, Tensor) else torch.as_tensor(np.asarray(v))
        if t.shape[0] % m:
            raise ValueError(f"feed '{name}' batch {t.shape[0]} is not divisible by num_microbatches {m}")
        for i, c in enumerate(torch.chunk(t, m, 0)):
            micro[i][name] = c
    per_mb = runner.run(micro, fetch_list or [])
    outs = []
    for j in range(len(fetch_list or [])):
        vals = [r[j] for r in per_mb]
        if any(v is None for v in vals):
            outs.append(None)
            continue
        vals = [v.detach() for v in vals]
        o = torch.stack(vals).mean(0) if vals[0].dim() == 0 else torch.cat(vals, 0)
        outs.append(o.cpu().numpy() if return_numpy else Tensor._wrap(o))
    return outs


class LarsMomentumOptimizer(Momentum):
    """reference incubate/optimizer/lars_momentum.py — momentum with the layer-wise LARS trust ratio
    lars_coeff * |w| / (|g| + lars_weight_decay * |w| + epsilon) (the ``lars_momentum`` kernel)."""

    def __init__(self, learning_rate, momentum, lars_coeff=0.001, lars_weight_decay=0.0005, parameter_list=None,
                 regularization=None, grad_clip=None, name=None, exclude_from_weight_decay=None, epsilon=0,
                 multi_precision=False, rescale_grad=1.0, parameters=None):
        params = parameters if parameters is not None else parameter_list
        super().__init__(learning_rate, momentum, params, weight_decay=regularization, grad_clip=grad_clip,
                         name=name)
        self._lars_coeff, self._lars_wd = float(lars_coeff), float(lars_weight_decay)
        self._exclude = list(exclude_from_weight_decay or [])
        self._lars_eps, self._rescale = float(epsilon), float(rescale_grad)
        self._multi_precision = multi_precision

    def _apply(self, pg):
        from ...ops.extra_ops import lars_momentum_

        lr = self.get_lr()
        for p, g in pg:
            wd = 0.0 if any(e in p.name for e in self._exclude) else self._lars_wd
            v = self._acc("velocity", p)
            mw = self._master(p)
            lars_momentum_(p._t, g._t, v, lr, mw, self._momentum, self._lars_coeff, (wd,), self._lars_eps,
                           mw is not None, self._rescale)


class DistributedFusedLamb(Lamb):
    """reference incubate/optimizer/distributed_fused_lamb.py — LAMB over one flat fp32 state.  With several
    ranks (``nproc_per_node`` of the data-parallel group) the flat gradient is reduce-scattered, each rank runs
    LAMB on its contiguous shard of every parameter's moments (per-parameter trust ratios from all-reduced
    squared norms) and the parameters are all-gathered; one rank is plain LAMB."""

    def __init__(self, learning_rate=0.001, lamb_weight_decay=0.01, beta1=0.9, beta2=0.999, epsilon=1e-6,
                 parameters=None, grad_clip=None, exclude_from_weight_decay_fn=None, clip_after_allreduce=True,
                 is_grad_scaled_by_nranks=True, alignment=128, use_master_param_norm=True,
                 gradient_accumulation_steps=1, use_master_acc_grad=True, nproc_per_node=None,
                 use_hierarchical_allreduce=False, name=None, group=None):
        super().__init__(learning_rate, lamb_weight_decay, beta1, beta2, epsilon, parameters, grad_clip,
                         exclude_from_weight_decay_fn, multi_precision=True, name=name)
        self._acc_steps = int(gradient_accumulation_steps)
        self._scaled_by_nranks = is_grad_scaled_by_nranks
        self._group = group
        self._acc_calls = 0

    def _world(self):
        import torch.distributed as tdist

        if not tdist.is_initialized():
            return 1, 0
        return tdist.get_world_size(self._group), tdist.get_rank(self._group)

    @torch.no_grad()
    def step(self):
        self._acc_calls += 1
        if self._acc_calls % self._acc_steps:
            return
        n, r = self._world()
        if n == 1:
            return super().step()
        return self._step_sharded(n, r)

    def _step_sharded(self, n, r):
        import torch.distributed as tdist

        ps = [p for p in self._parameter_list if p._t.grad is not None]
        if not ps:
            return
        dev = ps[0]._t.device
        sizes = [p._t.numel() for p in ps]
        total = sum(sizes)
        pad = (-total) % n
        flat_g = torch.cat([p._t.grad.reshape(-1).float() for p in ps] + [torch.zeros(pad, device=dev)])
        shard = flat_g.numel() // n
        g_sh = torch.empty(shard, device=dev)
        tdist.reduce_scatter_tensor(g_sh, flat_g, group=self._group)
        if self._scaled_by_nranks:
            g_sh.div_(n)
        flat_w = torch.cat([(self._master(p) if self._master(p) is not None else p._t.float()).reshape(-1)
                            for p in ps] + [torch.zeros(pad, device=dev)])
        w_sh = flat_w[r * shard:(r + 1) * shard].clone()
        st = self._accumulators
        if "flat_moment1" not in st or st["flat_moment1"].get("_", torch.empty(0)).numel() != shard:
            st["flat_moment1"]["_"] = torch.zeros(shard, device=dev)
            st["flat_moment2"]["_"] = torch.zeros(shard, device=dev)
        m1, m2 = st["flat_moment1"]["_"], st["flat_moment2"]["_"]
        self._step += 1
        m1.mul_(self._b1).add_(g_sh, alpha=1 - self._b1)
        m2.mul_(self._b2).addcmul_(g_sh, g_sh, value=1 - self._b2)
        upd = (m1 / (1 - self._b1 ** self._step)) / ((m2 / (1 - self._b2 ** self._step)).sqrt() + self._eps)
        # per-parameter weight decay and trust ratio: segment sums of squares over the shard, all-reduced
        bounds = torch.tensor([0] + sizes, device=dev).cumsum(0)
        idx = torch.arange(r * shard, (r + 1) * shard, device=dev)
        seg = torch.bucketize(idx, bounds[1:], right=True).clamp(max=len(ps))   # parameter index (len = padding)
        wd = torch.tensor([0.0 if (self._exclude is not None and self._exclude(p)) else self._wd for p in ps] + [0.0],
                          device=dev)
        upd = upd + wd[seg] * w_sh
        wn2 = torch.zeros(len(ps) + 1, device=dev).index_add_(0, seg, w_sh * w_sh)
        un2 = torch.zeros(len(ps) + 1, device=dev).index_add_(0, seg, upd * upd)
        both = torch.stack([wn2, un2])
        tdist.all_reduce(both, group=self._group)
        wn, un = both[0].sqrt(), both[1].sqrt()
        trust = torch.where((wn > 0) & (un > 0), wn / un, torch.ones_like(wn))
        w_sh.sub_(self.get_lr() * trust[seg] * upd)
        out = torch.empty_like(flat_w)
        tdist.all_gather_into_tensor(out, w_sh, group=self._group)
        off = 0
        for p, s in zip(ps, sizes):
            nw = out[off:off + s].view_as(p._t)
            mw = self._master(p)
            if mw is not None:
                mw.copy_(nw)
            p._t.copy_(nw.to(p._t.dtype))
            off += s
