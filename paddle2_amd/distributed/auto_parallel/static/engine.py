"""Static auto-parallel Engine (reference python/paddle/distributed/auto_parallel/static/engine.py: ``Engine``
``prepare`` / ``run`` / ``fit`` / ``evaluate`` / ``predict``).

``prepare`` records the serial forward (+ loss) Program for the input / label specs, completes it from the
annotations (parameters / feeds -> placements; with ``planner=True`` the 2-D weights' placements are chosen by the
MI355X cost model, ``cost_model.Planner``) and partitions it (``partitioner.DistributedProgram``).  Every sharded
Parameter then HOLDS ITS LOCAL SHARD (``param._t`` is replaced by the partitioner's leaf), so the user's own
optimizer steps the local shards and its accumulators are created at local shapes — the reference's
"optimizer ops run on the partitioned program" without a separate optimizer rewrite.  ``run`` executes one
step: partitioned forward, loss backward (conjugate collectives from the plan), optimizer step.
"""
from __future__ import annotations

import torch

from .completion import Completer, attr_from_placements
from .cost_model import CostModel, Planner
from .partitioner import DistributedProgram


class Engine:
    def __init__(self, model=None, loss=None, optimizer=None, metrics=None, mesh=None, annotations=None,
                 planner=False, strategy=None):
        self.model, self.loss, self.optimizer = model, loss, optimizer
        self.mesh = mesh
        self.annotations = dict(annotations or {})
        self.planner = planner
        self.strategy = strategy
        self._progs = {}
        self.history = []

    # ---------------------------------------------------------------- build
    def _record(self, inputs_spec, labels_spec, mode):
        from .... import static
        from ....static import graph as g

        prog = static.Program()
        was = g._state.static
        g._state.static = True
        try:
            with static.program_guard(prog, static.Program()):
                xs = [static.data(f"input_{i}", list(s.shape), s.dtype) for i, s in enumerate(inputs_spec)]
                ys = [static.data(f"label_{i}", list(s.shape), s.dtype) for i, s in enumerate(labels_spec or [])]
                out = self.model(*xs)
                loss = self.loss(out, *ys) if (mode != "predict" and self.loss is not None) else None
        finally:
            g._state.static = was
        return prog, out, loss

    def _plan_annotations(self, prog):
        if not self.planner:
            return self.annotations
        from ..api import Replicate, Shard

        opts = [[Replicate()], [Shard(0)], [Shard(1)]]
        cands = {p: opts for p in self.model.parameters() if p._t.dim() == 2 and p not in self.annotations}
        best, _ = Planner(prog, self.mesh, CostModel()).search(self.annotations, cands)
        return best

    def prepare(self, inputs_spec, labels_spec=None, mode="train"):
        """Record, complete and partition the forward+loss Program (train / eval) and the forward-only Program
        (predict) once, sharing one set of local parameter shards."""
        if self._progs:
            return self._progs.get("train" if mode == "eval" else mode)
        built = {}
        if labels_spec is not None and self.loss is not None:
            built["train"] = self._record(inputs_spec, labels_spec, "train")
        built["predict"] = self._record(inputs_spec, None, "predict")
        ann = self._plan_annotations(next(iter(built.values()))[0])
        self.chosen_annotations = ann
        leaves, objs = {}, {}
        for m, (prog, out, loss) in built.items():
            dp = DistributedProgram(prog, Completer(self.mesh).complete(prog, ann))
            for key in list(dp._local_params):
                if key in leaves:
                    dp._local_params[key] = leaves[key]
                else:
                    leaves[key], objs[key] = dp._local_params[key], dp._param_objs[key]
            self._progs[m] = (dp, out, loss)
        # parameters hold their local shards from here on (the optimizer then steps the shards)
        for key, leaf in leaves.items():
            p = objs[key]
            if tuple(p._t.shape) != tuple(leaf.shape):
                p._t = leaf
            else:  # replicated: keep the parameter's own storage as the leaf
                for dp, _, _ in self._progs.values():
                    dp._local_params[key] = p._t
        return self._progs.get("train" if mode == "eval" else mode)

    # ---------------------------------------------------------------- execution
    def run(self, inputs, labels=None, mode="train"):
        from ....framework.tensor import Tensor

        inputs = [x if isinstance(x, Tensor) else Tensor._wrap(torch.as_tensor(x)) for x in inputs]
        labels = [y if isinstance(y, Tensor) else Tensor._wrap(torch.as_tensor(y)) for y in (labels or [])]
        if not self._progs:
            from ....static import InputSpec

            self.prepare([InputSpec(list(x.shape), x.dtype) for x in inputs],
                         [InputSpec(list(y.shape), y.dtype) for y in labels] if labels else None, mode)
        dp, out, loss = self._progs["train" if mode == "eval" else mode]
        feed = {f"input_{i}": x for i, x in enumerate(inputs)}
        feed.update({f"label_{i}": y for i, y in enumerate(labels)})
        if mode == "predict":
            return dp.run(feed, [out])[0]
        (lval,) = dp.run(feed, [loss])
        if mode == "train":
            lval._t.backward()
            self.optimizer.step()
            self.optimizer.clear_grad()
        return Tensor._wrap(lval._t.detach())

    def fit(self, train_data, epochs=1, steps_per_epoch=None, log_freq=10, verbose=0):
        for _ in range(epochs):
            for step, batch in enumerate(train_data):
                if steps_per_epoch is not None and step >= steps_per_epoch:
                    break
                *xs, y = batch
                self.history.append(float(self.run(xs, [y], "train").numpy()))
        return self.history

    def evaluate(self, valid_data, steps=None):
        losses = []
        for step, batch in enumerate(valid_data):
            if steps is not None and step >= steps:
                break
            *xs, y = batch
            losses.append(float(self.run(xs, [y], "eval").numpy()))
        return {"loss": sum(losses) / max(len(losses), 1)}

    def predict(self, test_data, steps=None):
        outs = []
        for step, batch in enumerate(test_data):
            if steps is not None and step >= steps:
                break
            xs = batch if isinstance(batch, (list, tuple)) else [batch]
            outs.append(self.run(list(xs), None, "predict"))
        return outs


__all__ = ["Engine", "attr_from_placements"]
