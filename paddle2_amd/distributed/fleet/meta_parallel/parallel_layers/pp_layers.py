"""Pipeline model description (reference: fleet/meta_parallel/parallel_layers/pp_layers.py —
``LayerDesc`` :56, ``SharedLayerDesc`` :76, ``SegmentLayers`` :92, ``PipelineLayer`` :257).

A ``PipelineLayer`` is given the whole model as a list of ``LayerDesc`` (deferred constructors)
and plain callables; it segments the list into ``num_stages * num_virtual_pipeline_stages``
contiguous pieces (uniform by count, or balanced on a layer class with ``"layer:Name"``) and
builds ONLY the pieces this rank's pipeline stage owns (virtual stage ``v * S + s`` for chunk v),
so a 13B model's weights are never materialised on every GPU.
"""
from __future__ import annotations

import math
import re

import numpy as np

from .....nn.layer.layers import Layer
from .....nn.layer.common import LayerList


class LayerDesc:
    def __init__(self, layer_func, *inputs, **kwargs):
        self.layer_func = layer_func
        self.inputs = inputs
        self.kwargs = kwargs
        if not (isinstance(layer_func, type) and issubclass(layer_func, Layer)):
            raise TypeError("LayerDesc expects a Layer subclass")

    def build_layer(self):
        return self.layer_func(*self.inputs, **self.kwargs)

    def __repr__(self):
        return f"LayerDesc({self.layer_func.__name__})"


class SharedLayerDesc(LayerDesc):
    """A layer whose parameters are shared by several stages (e.g. tied embedding / LM head)."""

    def __init__(self, key, layer_func, forward_func=None, shared_weight_attr="weight", *inputs, **kwargs):
        super().__init__(layer_func, *inputs, **kwargs)
        self.layer_name = key
        self.forward_func = forward_func
        self.shared_weight_attr = shared_weight_attr


class SegmentLayers:
    def __init__(self, layers_desc, num_parts, method="uniform", num_virtual_pipeline_stage=None):
        self._layers_desc = layers_desc
        self.method = method
        self.num_parts = num_parts * (num_virtual_pipeline_stage or 1)
        self.num_items = len(layers_desc)
        assert self.num_items >= self.num_parts, "layer number should be greater than number of segments"

    def do_segment(self):
        if isinstance(self.method, list):
            return self.method
        if self.method == "uniform":
            return self.uniform(self.num_items, self.num_parts)
        if self.method.startswith("layer:"):
            name = self.method.split(":", 1)[1]
            weights = [1 if self._match(d, name) else 0 for d in self._layers_desc]
            total = sum(weights)
            assert total >= self.num_parts, f"only {total} '{name}' layers for {self.num_parts} segments"
            per = self.uniform(total, self.num_parts)
            # cut points at the per[i]-th matching layer; leading non-matching layers go to part 0
            idx = [i for i, w in enumerate(weights) if w]
            res = [0] + [idx[per[i]] for i in range(1, self.num_parts)] + [self.num_items]
            return res
        raise ValueError(f"unknown seg_method {self.method}")

    @staticmethod
    def _match(desc, name):
        f = desc.layer_func if isinstance(desc, LayerDesc) else type(desc)
        return re.search(name, getattr(f, "__name__", "")) is not None

    @staticmethod
    def uniform(num_items, num_parts):
        res = [0] * (num_parts + 1)
        chunk, extra = divmod(num_items, num_parts)
        for i in range(1, num_parts + 1):
            res[i] = res[i - 1] + chunk + (1 if i - 1 < extra else 0)
        res[-1] = num_items
        return res


class _Chunk(Layer):
    """One virtual stage's contiguous run of layers/callables."""

    def __init__(self, items):
        super().__init__()
        self._items = []
        self.run_function = LayerList()
        for it in items:
            if isinstance(it, Layer):
                self.run_function.append(it)
            self._items.append(it)

    def forward(self, x):
        for f in self._items:
            x = f(*x) if isinstance(x, tuple) else f(x)
        return x


class PipelineLayer(Layer):
    def __init__(self, layers, num_stages=None, topology=None, loss_fn=None, seg_method="uniform",
                 recompute_interval=0, recompute_ctx=None, num_virtual_pipeline_stages=None):
        super().__init__()
        from .... import fleet

        if num_stages is None and topology is None:
            hcg = fleet.get_hybrid_communicate_group()
            topology = hcg.topology() if hcg is not None else None
        if topology is not None:
            self._num_stages = topology.get_dim("pipe")
            hcg = fleet.get_hybrid_communicate_group()
            self._stage_id = hcg.get_stage_id() if hcg is not None else 0
        else:
            self._num_stages = num_stages
            self._stage_id = 0
        self._topo = topology
        self._loss_fn = loss_fn
        self._recompute_interval = recompute_interval
        self._num_virtual_pipeline_stages = num_virtual_pipeline_stages or 1
        self._layers_desc = list(layers)
        seg = SegmentLayers(self._layers_desc, self._num_stages, seg_method, self._num_virtual_pipeline_stages)
        self.segment_parts = seg.do_segment()
        S, V = self._num_stages, self._num_virtual_pipeline_stages
        self.shared_layers = {}
        self.shared_weight_attrs = {}
        self._shared_owners = {}  # key -> sorted list of stages using it
        for vs in range(S * V):
            for d in self._layers_desc[self.segment_parts[vs]:self.segment_parts[vs + 1]]:
                if isinstance(d, SharedLayerDesc):
                    self._shared_owners.setdefault(d.layer_name, set()).add(vs % S)
        self._model_chunks = LayerList()
        self._chunk_vstages = []
        for v in range(V):
            vs = v * S + self._stage_id
            items = []
            for d in self._layers_desc[self.segment_parts[vs]:self.segment_parts[vs + 1]]:
                items.append(self._build(d))
            self._model_chunks.append(_Chunk(items))
            self._chunk_vstages.append(vs)
        self.run_function = self._model_chunks[0].run_function if V == 1 else None

    def _build(self, d):
        if isinstance(d, SharedLayerDesc):
            if d.layer_name not in self.shared_layers:
                self.shared_layers[d.layer_name] = d.build_layer()
                self.shared_weight_attrs[d.layer_name] = d.shared_weight_attr
            layer = self.shared_layers[d.layer_name]
            if d.forward_func is None:
                return layer
            ff = d.forward_func

            def run(*x, _l=layer, _f=ff):
                return _f(_l, *x)

            return run
        if isinstance(d, LayerDesc):
            return d.build_layer()
        return d

    # ------------------------------------------------------------------ API
    def get_stage_from_index(self, layer_idx):
        for vs in range(len(self.segment_parts) - 1):
            if self.segment_parts[vs] <= layer_idx < self.segment_parts[vs + 1]:
                return vs % self._num_stages
        raise IndexError(layer_idx)

    # ------------------------------------------------------------------ pipeline-agnostic checkpoints
    def _global_key_map(self):
        """local state-dict key -> "layers.{global layer index}.{param}" (shared layers keep
        "shared_layers.{name}.*"), so a checkpoint does not depend on the pp / vpp split."""
        m = {}
        for c, vs in enumerate(self._chunk_vstages):
            li = 0
            for g in range(self.segment_parts[vs], self.segment_parts[vs + 1]):
                item = self._model_chunks[c]._items[g - self.segment_parts[vs]]
                if isinstance(item, Layer) and not isinstance(self._layers_desc[g], SharedLayerDesc):
                    for k in item.state_dict():
                        m[f"_model_chunks.{c}.run_function.{li}.{k}"] = f"layers.{g}.{k}"
                        if self.run_function is not None and c == 0:  # the V == 1 alias of chunk 0
                            m[f"run_function.{li}.{k}"] = f"layers.{g}.{k}"
                if isinstance(item, Layer):
                    li += 1
        return m

    def global_state_dict(self):
        km = self._global_key_map()
        return {km.get(k, k): v for k, v in self.state_dict().items()}

    def set_global_state_dict(self, sd):
        km = self._global_key_map()
        local = {lk: sd[gk] for lk, gk in km.items() if gk in sd}
        local.update({k: v for k, v in sd.items() if k in self.state_dict() and k not in km})
        return self.set_state_dict(local)

    def get_num_virtual_stages(self):
        return self._num_virtual_pipeline_stages

    def get_model_chunks(self):
        return list(self._model_chunks)

    def is_first_vstage(self, chunk_id):
        return self._chunk_vstages[chunk_id] == 0

    def is_last_vstage(self, chunk_id):
        return self._chunk_vstages[chunk_id] == self._num_stages * self._num_virtual_pipeline_stages - 1

    def shared_params(self):
        """[(key, param, stages_sharing_it)] for SharedLayerDesc weights used on >1 stage."""
        out = []
        for k, layer in self.shared_layers.items():
            stages = sorted(self._shared_owners[k])
            if len(stages) > 1:
                out.append((k, getattr(layer, self.shared_weight_attrs[k]), stages))
        return out

    def forward(self, input, chunk_id=None):
        if chunk_id is None:
            assert self._num_virtual_pipeline_stages == 1
            chunk_id = 0
        chunk = self._model_chunks[chunk_id]
        if self._recompute_interval > 0 and self.training:
            from ...recompute import recompute

            items = chunk._items
            x = input
            for s in range(0, len(items), self._recompute_interval):
                seg = items[s:s + self._recompute_interval]

                def f(*xs, _seg=seg):
                    y = xs if len(xs) > 1 else xs[0]
                    for fn in _seg:
                        y = fn(*y) if isinstance(y, tuple) else fn(y)
                    return y

                x = recompute(f, *(x if isinstance(x, tuple) else (x,)))
            return x
        return chunk(input)
