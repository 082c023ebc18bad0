#!/usr/bin/env python
"""ResNet50 bf16 data-parallel training benchmark (BASELINE.json config 2: "ResNet50 bf16 Fleet DP on
1→8 MI355X (fused_adamw kernel, RCCL allreduce)").

One step = forward + backward (bucketed RCCL all-reduce overlapped with backward through the
DataParallel reducer) + fused multi-tensor AdamW with fp32 master weights.  Activations are
channels-last (NHWC), the layout MIOpen's bf16 convolutions are fastest in; BatchNorm runs in fp32
(AMP O2 keeps norm layers fp32).  Synthetic 224x224 images and random labels, random-init weights.

    python scripts/bench_resnet50.py --steps 20 --warmup 5
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 scripts/bench_resnet50.py
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _find_db_setup(args):
    """Point MIOpen's user db at a scratch copy of the seed (before the first convolution initialises MIOpen)."""
    import shutil
    import tempfile

    if "MIOPEN_USER_DB_PATH" in os.environ:
        return
    db = tempfile.mkdtemp(prefix="miopen_db_")
    if args.find_db and os.path.isdir(args.find_db):
        for f in os.listdir(args.find_db):
            if f.endswith(".txt"):
                shutil.copy(os.path.join(args.find_db, f), db)
    os.environ["MIOPEN_USER_DB_PATH"] = db


def _find_db_save(dst):
    import shutil

    os.makedirs(dst, exist_ok=True)
    src = os.environ["MIOPEN_USER_DB_PATH"]
    for f in os.listdir(src):
        if f.endswith(".txt"):
            shutil.copy(os.path.join(src, f), dst)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256, help="images per GPU per step")
    ap.add_argument("--data-format", default="NHWC", choices=["NHWC", "NCHW"])
    ap.add_argument("--dtype", default="bfloat16", choices=["bfloat16", "float32"])
    ap.add_argument("--exhaustive-search", type=int, default=1, choices=[0, 1],
                    help="FLAGS_cudnn_exhaustive_search: MIOpen Find per conv shape (the reference's ResNet recipes "
                         "set it); 0 = MIOpen's immediate-mode heuristic")
    ap.add_argument("--find-db", default=os.path.join(ROOT, "tuning", "miopen"),
                    help="MIOpen user find-db seed directory (text records of the solver Find chose per shape, made "
                         "by an earlier --save-find-db run): copied to a scratch MIOPEN_USER_DB_PATH so a fresh box "
                         "skips the search ('' = search from scratch)")
    ap.add_argument("--save-find-db", default="", help="copy the user find-db here after the run")
    args = ap.parse_args()
    _find_db_setup(args)

    import torch

    import paddle2_amd as paddle
    from paddle2_amd.distributed import fleet
    from paddle2_amd.vision.models import resnet50

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    paddle.set_flags({"FLAGS_cudnn_exhaustive_search": bool(args.exhaustive_search)})
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": world, "mp_degree": 1, "pp_degree": 1, "sharding_degree": 1}
    fleet.init(is_collective=True, strategy=strategy)
    paddle.seed(0)

    model = resnet50(data_format=args.data_format)
    opt = paddle.optimizer.AdamW(learning_rate=1e-3, parameters=model.parameters(), weight_decay=0.05,
                                 multi_precision=True)
    if args.dtype == "bfloat16":
        model, opt = paddle.amp.decorate(model, opt, level="O2", dtype="bfloat16")
    if world > 1:
        model = fleet.distributed_model(model)
        opt = fleet.distributed_optimizer(opt)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    dt = torch.bfloat16 if args.dtype == "bfloat16" else torch.float32
    shape = (args.batch, 224, 224, 3) if args.data_format == "NHWC" else (args.batch, 3, 224, 224)
    gen = torch.Generator(device=dev).manual_seed(rank)
    x = paddle.Tensor._wrap(torch.randn(shape, generator=gen, device=dev).to(dt))
    y = paddle.Tensor._wrap(torch.randint(0, 1000, (args.batch,), generator=gen, device=dev))
    loss_fn = paddle.nn.CrossEntropyLoss()

    def step():
        logits = model(x)
        loss = loss_fn(logits.astype("float32"), y)
        loss.backward()
        opt.step()
        opt.clear_grad()
        return loss

    for i in range(args.warmup):
        tw = time.perf_counter()
        loss = step()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if rank == 0:   # progress (MIOpen Find can spend minutes on the first step's shapes)
            print(f"[resnet50] warmup step {i}: {time.perf_counter() - tw:.1f} s", file=sys.stderr, flush=True)
    from paddle2_amd.distributed import collective as C

    def sync():
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        if world > 1:
            C.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()

    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        loss = step()
    sync()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    ips = args.batch * world * args.steps / elapsed
    if rank == 0:
        print(json.dumps({
            "metric": "images/sec (whole node) ResNet50 Fleet DP",
            "value": round(ips, 1), "unit": "images/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 2), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "bf16" if dt == torch.bfloat16 else "fp32",
            "data": "synthetic 224x224 images, random labels; random-init weights",
            "config": {"model": "resnet50", "global_batch": args.batch * world, "batch_per_gpu": args.batch,
                       "data_format": args.data_format, "parallelism": f"dp{world}"},
            "final_loss": round(float(loss), 4),
            "exhaustive_search": bool(args.exhaustive_search),
            "peak_mem_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1) if torch.cuda.is_available() else None,
        }), flush=True)
        from paddle2_amd.ops import conv_gemm as CG

        for k, v in sorted(CG._ROUTE.items(), key=str):
            print("conv routes:", k[0], "x", list(k[1]), "w", list(k[2]), "stride", list(k[3]),
                  "native" if v else "miopen", file=sys.stderr)
        if args.save_find_db:
            _find_db_save(args.save_find_db)
    if world > 1:
        C.destroy_process_group()


if __name__ == "__main__":
    main()
