"""Offline re-partitioning of pipeline-parallel checkpoints between pp degrees (reference:
python/paddle/distributed/fleet/utils/pp_parallel_adaptor.py — ParallelConfig, PipeLineModelAdaptor).

Layout: one directory per rank, ``{root}/mp_{i:02d}_sharding_{j:02d}_pp_{k:02d}/model.pdparams``, whose keys are
pipeline-agnostic (``PipelineLayer.global_state_dict``: ``layers.{global index}.*`` and ``shared_layers.*``).
For every (mp, sharding) coordinate the adaptor merges the source stages' dicts, re-splits the layer indices
uniformly over the destination pp degree (``segment_method="layer"``: transformer layers balanced, leading /
trailing non-transformer layers stay with the first / last stage) and writes the destination directories;
shared layers go to every destination stage that holds their first or last use (first and last stage).
No model is instantiated and nothing is executed from the files beyond the framework's restricted loader.
"""
from __future__ import annotations

import argparse
import os
import re

from ....framework.io import load as _load
from ....framework.io import save as _save

_LAYER = re.compile(r"^layers\.(\d+)\.(.+)$")


class ParallelConfig:
    def __init__(self, mp: int, pp: int, vpp: int = 1, sharding: int = 1):
        self.mp, self.pp, self.vpp, self.sharding = int(mp), int(pp), int(vpp), int(sharding)

    def pipe_parallel_group(self, i: int, j: int):
        return [(i, j, k) for k in range(self.pp)]


def _dir(root, i, j, k):
    return os.path.join(root, f"mp_{i:02d}_sharding_{j:02d}_pp_{k:02d}")


def _uniform(n, parts):
    chunk, extra = divmod(n, parts)
    cuts = [0]
    for p in range(parts):
        cuts.append(cuts[-1] + chunk + (1 if p < extra else 0))
    return cuts


class PipeLineModelAdaptor:
    def __init__(self, src_parallel_config: ParallelConfig, dst_parallel_config: ParallelConfig,
                 transformer_layer_num: int, segment_method: str = "layer"):
        if src_parallel_config.mp != dst_parallel_config.mp or \
                src_parallel_config.sharding != dst_parallel_config.sharding:
            raise ValueError("pp adaptor re-splits pipeline stages only (mp / sharding degrees must match)")
        self.src, self.dst = src_parallel_config, dst_parallel_config
        self.transformer_layer_num = int(transformer_layer_num)
        self.segment_method = segment_method

    @staticmethod
    def extract_layers(path):
        sd = _load(os.path.join(path, "model.pdparams"))
        layers, shared = {}, {}
        for k, v in sd.items():
            m = _LAYER.match(k)
            if m:
                layers.setdefault(int(m.group(1)), {})[m.group(2)] = v
            else:
                shared[k] = v
        return layers, shared

    def segment(self, layer_ids, parts):
        """Cut the sorted global layer ids into ``parts`` stages."""
        ids = sorted(layer_ids)
        if self.segment_method == "uniform" or len(ids) <= self.transformer_layer_num:
            cuts = _uniform(len(ids), parts)
            return [ids[cuts[p]:cuts[p + 1]] for p in range(parts)]
        # "layer": balance the transformer layers (the middle run), extras ride with the first / last stage
        head = (len(ids) - self.transformer_layer_num) // 2
        body = ids[head:head + self.transformer_layer_num]
        cuts = _uniform(len(body), parts)
        segs = [body[cuts[p]:cuts[p + 1]] for p in range(parts)]
        segs[0] = ids[:head] + segs[0]
        segs[-1] = segs[-1] + ids[head + self.transformer_layer_num:]
        return segs

    def apply(self, src_model_path: str, dst_model_path: str):
        for i in range(self.src.mp):
            for j in range(self.src.sharding):
                layers, shared = {}, {}
                for (_, _, k) in self.src.pipe_parallel_group(i, j):
                    lyr, sh = self.extract_layers(_dir(src_model_path, i, j, k))
                    for g, params in lyr.items():
                        if g in layers and layers[g].keys() != params.keys():
                            raise ValueError(f"layer {g} appears on two stages with different parameters")
                        layers[g] = params
                    for kk, v in sh.items():
                        shared.setdefault(kk, v)  # tied copies are equal; keep the first stage's
                segs = self.segment(layers.keys(), self.dst.pp)
                for k, seg in enumerate(segs):
                    out = {}
                    for g in seg:
                        out.update({f"layers.{g}.{n}": v for n, v in layers[g].items()})
                    if k in (0, self.dst.pp - 1):
                        out.update(shared)
                    d = _dir(dst_model_path, i, j, k)
                    os.makedirs(d, exist_ok=True)
                    _save(out, os.path.join(d, "model.pdparams"))


def parse_args(argv=None):
    p = argparse.ArgumentParser("pp_parallel_adaptor")
    p.add_argument("--src_path", required=True)
    p.add_argument("--dst_path", required=True)
    p.add_argument("--src_mp", type=int, default=1)
    p.add_argument("--dst_mp", type=int, default=1)
    p.add_argument("--src_pp", type=int, required=True)
    p.add_argument("--dst_pp", type=int, required=True)
    p.add_argument("--src_vp", type=int, default=1)
    p.add_argument("--dst_vp", type=int, default=1)
    p.add_argument("--sharding", type=int, default=1)
    p.add_argument("--transformer_layer_num", type=int, required=True)
    p.add_argument("--segment_method", default="layer")
    return p.parse_args(argv)


def adaptor_from_args(args):
    src = ParallelConfig(args.src_mp, args.src_pp, args.src_vp, args.sharding)
    dst = ParallelConfig(args.dst_mp, args.dst_pp, args.dst_vp, args.sharding)
    return PipeLineModelAdaptor(src, dst, args.transformer_layer_num, args.segment_method)


def main(argv=None):
    args = parse_args(argv)
    adaptor_from_args(args).apply(args.src_path, args.dst_path)


if __name__ == "__main__":
    main()
