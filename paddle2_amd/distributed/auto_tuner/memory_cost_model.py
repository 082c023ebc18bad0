"""Memory estimation tool for ``tuner_cfg['memory_estimation_tool']`` (reference:
python/paddle/distributed/auto_tuner/memory_cost_model.py, whose get_model_memory_usage is left to the
user).  Prints the analytical per-GPU peak of ``cost_model.estimate_memory_gb`` in MiB, so the prune
rule can compare it with ``max_mem_usage`` GiB:

    python -m paddle2_amd.distributed.auto_tuner.memory_cost_model --dp_degree 1 --mp_degree 2 ...
"""
from __future__ import annotations

from argparse import ArgumentParser

from .cost_model import estimate_memory_gb


def _bool(v):
    return str(v).lower() in ("1", "true", "yes")


def parse_arguments(argv=None):
    ap = ArgumentParser()
    for k in ("dp_degree", "mp_degree", "pp_degree", "vpp_degree", "sharding_degree", "sharding_stage",
              "micro_batch_size"):
        ap.add_argument(f"--{k}", type=int, required=True)
    ap.add_argument("--use_recompute", type=_bool, required=True)
    ap.add_argument("--recompute_granularity", type=str, default="None")
    for k in ("hidden_size", "num_attention_heads", "num_layers", "vocab_size", "intermediate_size",
              "num_key_value_heads"):
        ap.add_argument(f"--{k}", type=int, default=None)
    ap.add_argument("--seq_length", "--max_sequence_length", dest="seq_length", type=int, default=4096)
    return ap.parse_args(argv)


def get_model_memory_usage(args):
    model = {k: getattr(args, k) for k in ("hidden_size", "num_attention_heads", "num_layers", "vocab_size",
                                           "intermediate_size", "num_key_value_heads", "seq_length")
             if getattr(args, k) is not None}
    cfg = {k: getattr(args, k) for k in ("dp_degree", "mp_degree", "pp_degree", "vpp_degree", "sharding_degree",
                                         "sharding_stage", "micro_batch_size", "use_recompute")}
    cfg["recompute_granularity"] = None if args.recompute_granularity in ("None", "") else args.recompute_granularity
    return estimate_memory_gb(model, cfg) * 1024


if __name__ == "__main__":
    print(round(get_model_memory_usage(parse_arguments()), 2))
