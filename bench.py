#!/usr/bin/env python
"""Flagship benchmark: Llama-2-7B pretraining step, Fleet sharding stage 3, bf16, synthetic data.

Metric (BASELINE.json): tokens/sec for the whole node, Llama-2-7B Fleet sharding-3 bf16 at
1/2/4/8 MI355X.  Weak scaling: every rank trains ``--micro-batch`` sequences of ``--seq-len`` tokens
per step, so global_batch = micro_batch * N.

Launch:  python bench.py --gpus N --steps K --warmup W
           (N > 1 without WORLD_SIZE: this process starts N ranks through the in-tree launcher
            ``python -m paddle2_amd.distributed.launch`` — one process per GPU, RCCL — and exits with
            their status; only global rank 0 prints the JSON line)
         python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
             --master-port P bench.py --gpus N --steps K --warmup W

Every N (including N = 1) runs the same code path: the model is wrapped by
``group_sharded_parallel(level="p_g_os")`` (stage 3: flat per-layer units, all-gather prefetch,
fp32 main-grad accumulation straight from the weight-gradient GEMMs, reduce-scatter, sharded fused
AdamW).  The timed region is exactly K full steps (forward + backward + grad reduce-scatter +
global-norm clip + fused AdamW with fp32 master weights), bracketed by barrier +
torch.cuda.synchronize(); the reported time is the max over ranks.  Data: a fresh batch of synthetic
token ids (uniform over the 32000-token vocab) every step, pre-generated on the device before the
timed region; random-init weights of the exact Llama-2-7B architecture.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))


def parse(argv=None):
    ap = argparse.ArgumentParser(
        formatter_class=argparse.RawDescriptionHelpFormatter,
        epilog="""BASELINE.json configs on one 8-GPU node (T = torchrun --nnodes=1 --nproc-per-node 8 \\
    --master-addr 127.0.0.1 --master-port 29500; or drop T and let --gpus 8 self-launch):
  3  Llama-2 7B Fleet sharding-3 bf16 (the headline):
       T bench.py --gpus 8
  4  Llama-2 13B TP=2 x PP=4 hybrid (1F1B, Column/RowParallelLinear over xGMI):
       T bench.py --gpus 8 --model llama2-13b --mp 2 --pp 4 --micro-batch 1 --seq-len 4096
       (4 x pp = 16 micro-batches of 1 x 4096 per step by default: --accumulate-steps)
  5  GPT-3 13B fp8 MFMA + sequence-parallel + sharding-3 (TP=2 x sharding 4):
       T bench.py --gpus 8 --model gpt3-13b --fp8 --mp 2 --sp --seq-len 2048 --micro-batch 4
  2  ResNet50 bf16 DP: scripts/bench_resnet50.py""")
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--seq-len", type=int, default=4096)
    ap.add_argument("--micro-batch", type=int, default=8,
                    help="sequences per GPU per step (8 x 4096 tokens fits one 288 GB MI355X)")
    ap.add_argument("--model", default="llama2-7b",
                    choices=["llama2-7b", "llama2-13b", "tiny", "gpt3-13b", "gpt3-6.7b", "gpt3-1.3b", "gpt3-tiny"])
    ap.add_argument("--fp8", action="store_true", help="GPT configs: fp8 (e4m3/e5m2 delayed scaling) linears")
    ap.add_argument("--layers", type=int, default=None, help="DEBUG ONLY: override layer count (invalid for the metric)")
    ap.add_argument("--sharding-stage", type=int, default=3, choices=[0, 1, 2, 3],
                    help="0 = no sharding wrapper (DEBUG: not the metric's code path)")
    ap.add_argument("--mp", type=int, default=1, help="tensor-parallel degree (Column/RowParallelLinear)")
    ap.add_argument("--pp", type=int, default=1, help="pipeline-parallel degree (Llama: LlamaForCausalLMPipe)")
    ap.add_argument("--vpp", type=int, default=1, help="virtual pipeline stages per rank (interleaved 1F1B)")
    ap.add_argument("--pp-schedule", default="1F1B", choices=["1F1B", "FThenB", "VPP", "ZBH1"])
    ap.add_argument("--sp", action="store_true", help="sequence parallelism inside the TP group (needs --mp > 1)")
    ap.add_argument("--dp", type=int, default=1, help="data-parallel degree (the rest of the world is sharding)")
    ap.add_argument("--recompute", action="store_true")
    ap.add_argument("--accumulate-steps", type=int, default=1,
                    help="micro-batches per optimizer step (gradient accumulation into the fp32 main grads)")
    ap.add_argument("--profile-steps", type=int, default=0)
    ap.add_argument("--gemm-autotune", default="auto", choices=["auto", "tune", "off"],
                    help="hipBLASLt solution cache (tuning/gemm_gfx950.csv): auto = use it if present")
    ap.add_argument("--expect-pg", default="auto", choices=["auto", "pdrccl", "c10d", "gloo", "any"],
                    help="process group the run must be on (auto: pdrccl on GPUs unless PADDLE2_AMD_PG opts out, gloo "
                         "on CPU); a mismatch — e.g. a failed start-up canary that fell back to c10d — exits 3")
    ap.add_argument("--allow-pg-fallback", action="store_true", help="accept a fallen-back process group (= any)")
    ap.add_argument("--hang-guard-s", type=float, default=0.0,
                    help="bound on the timed region (0: max(300 s, 20 x the measured warm-up step time x steps)); "
                         "past it every rank dumps its last collective per group and exits 124")
    ap.add_argument("--comm-probe-mb", type=float, default=-1.0,
                    help="N > 1: per-rank MB of an all-gather / reduce-scatter / all-reduce probe on the world group "
                         "after the warm-up (bus bandwidth in the metric line: the communicator's own speed beside the "
                         "scaling curve); -1 = 32 MB on GPUs, 1 MB on CPU; 0 = off")
    ap.add_argument("--gemm-route", default="static", choices=["static", "measure"],
                    help="bf16 Linear GEMM backend per shape: static = the per-pass table (ops/gemm.py: the native "
                         "kernels), measure = time native vs hipBLASLt per (pass, M, N, K) once (incubate/autotune.py "
                         "route).  GPT-3 13B: static 10,893 vs measure 10,860 tokens/s with the tail split-K "
                         "(profiles/r4_gemm_tail_splitk.md)")
    return ap.parse_args(argv)


def _self_launch(args) -> int:
    """Start args.gpus ranks (one per GPU) via the in-tree launcher; never exec (GPU not touched here)."""
    log_dir = tempfile.mkdtemp(prefix="bench_launch_")
    cmd = [sys.executable, "-m", "paddle2_amd.distributed.launch", "--nproc_per_node", str(args.gpus),
           "--log_dir", log_dir, os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env, cwd=ROOT)


def expected_pg(world, on_gpu, native_enabled, want="auto", requested=None):
    """The process-group backend a run of ``world`` ranks must report (None: no requirement).  ``requested``: an
    explicitly chosen backend (PADDLE_DISTRI_BACKEND) — gloo / mpi then run on gloo by the user's choice."""
    if world <= 1 or want == "any":
        return None
    if want != "auto":
        return want
    if not on_gpu or (requested or "").lower() in ("gloo", "mpi"):
        return "gloo"
    return "pdrccl" if native_enabled else "c10d"


def pg_problem(status, expect):
    """Error text when the job's process group is not the expected one (a silent fallback), else None."""
    if expect is None or status.get("backend") == expect:
        return None
    return (f"process group is {status.get('backend')!r}, expected {expect!r} (start-up canary verdicts: "
            f"{status.get('canary')}); refusing to report a number from a fallen-back communicator "
            "(--allow-pg-fallback / --expect-pg any to accept)")


def _hang_report(guard_s):
    """Printed by every rank when the timed region outlives its guard: the communicator state and the latest
    collective of each process group, then a non-zero exit (no re-exec; the launcher tears the job down)."""
    rep = {"error": "bench timed region exceeded its guard", "guard_s": round(guard_s, 1),
           "rank": int(os.environ.get("RANK", "0"))}
    try:
        from paddle2_amd.distributed import collective as C

        rep["pg"] = C.pg_status()
    except Exception as e:  # noqa: BLE001 - diagnostics only
        rep["pg"] = repr(e)
    try:
        from paddle2_amd.distributed import rccl_pg

        rep["last_ops"] = rccl_pg.last_ops()
    except Exception as e:  # noqa: BLE001
        rep["last_ops"] = repr(e)
    try:
        from paddle2_amd.distributed import watchdog

        rep["watchdog_timeouts"] = watchdog.check_once(0.0)
    except Exception as e:  # noqa: BLE001
        rep["watchdog_timeouts"] = repr(e)
    print(json.dumps(rep, default=str), file=sys.stderr, flush=True)
    sys.stdout.flush()
    os._exit(124)


def comm_probe(world, mb, on_gpu):
    """{op: bus GB/s} of an all-gather, reduce-scatter and all-reduce of ``mb`` MB per rank (bf16) on the world group
    (fleet.collective_perf's timing, nccl-tests bus conventions), or None for one rank / mb == 0."""
    if world <= 1 or mb == 0:
        return None
    import torch

    from paddle2_amd.distributed import collective as C
    from paddle2_amd.distributed.fleet.collective_perf import perf_one

    if mb < 0:
        mb = 32.0 if on_gpu else 1.0
    nbytes = int(mb * 2**20)
    out = {"mb_per_rank": mb}
    for op in ("allgather", "reduce_scatter", "allreduce"):
        # all-gather sends its input to every peer; reduce-scatter / all-reduce take the full buffer
        r = perf_one(op, nbytes if op == "allgather" else nbytes * world, C._get_default_group(),
                     round=5 if on_gpu else 2, dtype=torch.bfloat16)
        out[op + "_busbw_GBps"] = float(f'{r["busbw_GBs"]:.3g}')   # 3 significant: a loaded gloo host is < 0.05 GB/s
        out[op + "_ms"] = round(r["time_ms"], 3)
    return out


def main():
    args = parse()
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(_self_launch(args))
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"error: WORLD_SIZE={world} but --gpus={args.gpus}", file=sys.stderr)
        sys.exit(2)
    rank = int(os.environ.get("RANK", "0"))

    import torch

    import paddle2_amd as paddle
    from paddle2_amd.distributed import fleet
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM, llama_flops_per_token

    if args.gemm_autotune != "off" and torch.cuda.is_available():
        from paddle2_amd.incubate import autotune

        if args.gemm_autotune == "tune" or os.path.exists(autotune.DEFAULT_GEMM_CACHE):
            autotune.enable_gemm_autotune(tuning=args.gemm_autotune == "tune")
    if args.gemm_route == "measure":
        if torch.cuda.is_available():
            from paddle2_amd.incubate import autotune

            autotune.enable_routing_autotune(os.path.join(tempfile.gettempdir(), f"gemm_route_{os.getpid()}.json"))

    mp, pp, vpp, dp = args.mp, args.pp, args.vpp, args.dp
    if world % (mp * pp * dp):
        print(f"error: world {world} is not a multiple of mp {mp} x pp {pp} x dp {dp}", file=sys.stderr)
        sys.exit(2)
    sh = world // (mp * pp * dp)   # the rest of the world shards the model / optimizer state
    if args.sp and mp == 1:
        print("error: --sp needs --mp > 1", file=sys.stderr)
        sys.exit(2)
    if pp > 1 and (args.model.startswith("gpt3") or sh > 1):
        print("error: --pp runs the Llama pipeline form without sharding (mp x pp x dp == world)", file=sys.stderr)
        sys.exit(2)
    if dp > 1 and sh > 1 and args.sharding_stage > 0:
        print("error: --dp > 1 with sharding: use --dp world (pure DP, --sharding-stage 0) or --dp 1", file=sys.stderr)
        sys.exit(2)
    acc = max(1, args.accumulate_steps)
    if pp > 1 and args.accumulate_steps == 1:
        acc = 4 * pp * vpp   # micro-batches per step: 1F1B bubble (pp-1)/(acc+pp-1) = 16 % at pp 4
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": dp, "mp_degree": mp, "pp_degree": pp, "sharding_degree": sh}
    if pp > 1:
        strategy.pipeline_configs = {"accumulate_steps": acc, "micro_batch_size": args.micro_batch,
                                     "schedule_mode": args.pp_schedule if vpp == 1 else "VPP"}
    fleet.init(is_collective=True, strategy=strategy)
    from paddle2_amd.distributed import collective as C

    # what actually runs the collectives: a fallback (failed canary -> c10d, or gloo) must not yield a silent number
    pgs = C.pg_status()
    native_on = False
    if torch.cuda.is_available():
        from paddle2_amd.distributed import rccl_pg

        native_on = rccl_pg.enabled()
    want = "any" if args.allow_pg_fallback else args.expect_pg
    err = pg_problem(pgs, expected_pg(world, torch.cuda.is_available(), native_on, want,
                                      os.environ.get("PADDLE_DISTRI_BACKEND")))
    if err:
        print(f"error: {err}", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(3)
    paddle.seed(1234)  # same init on every rank (stage 3 shards one replica)

    is_gpt = args.model.startswith("gpt3")
    extra = {"tensor_parallel_degree": mp, "sequence_parallel": bool(args.sp)}
    if is_gpt:
        from paddle2_amd.models import GPTConfig, GPTForCausalLM, gpt_flops_per_token

        cfg = {"gpt3-13b": GPTConfig.gpt3_13b, "gpt3-6.7b": GPTConfig.gpt3_6_7b, "gpt3-1.3b": GPTConfig.gpt3_1_3b,
               "gpt3-tiny": GPTConfig.tiny}[args.model](use_fp8=args.fp8, **extra)
    elif args.model == "llama2-7b":
        cfg = LlamaConfig.llama2_7b(**extra)
    elif args.model == "llama2-13b":
        cfg = LlamaConfig.llama2_13b(**extra)
    else:
        cfg = LlamaConfig.tiny(**extra)
    cfg.max_position_embeddings = max(cfg.max_position_embeddings, args.seq_len)
    if args.layers:
        cfg.num_hidden_layers = args.layers
    cfg.recompute = args.recompute

    if pp > 1:
        from paddle2_amd.models import LlamaForCausalLMPipe

        model = LlamaForCausalLMPipe(cfg, num_virtual_pipeline_stages=vpp if vpp > 1 else None)
    else:
        model = GPTForCausalLM(cfg) if is_gpt else LlamaForCausalLM(cfg)
    decay = {p.name for n, p in model.named_parameters() if "norm" not in n}
    opt = paddle.optimizer.AdamW(learning_rate=3e-4, beta1=0.9, beta2=0.95, epsilon=1e-8,
                                 parameters=model.parameters(), weight_decay=0.1,
                                 apply_decay_param_fun=lambda n: n in decay,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0), multi_precision=True)
    if pp > 1 or (mp > 1 and args.sharding_stage == 0) or dp > 1 and args.sharding_stage == 0:
        # hybrid TP x PP (x DP): the fleet wrappers (PipelineParallel 1F1B / TensorParallel, HybridParallelOptimizer)
        model = fleet.distributed_model(model)
        opt = fleet.distributed_optimizer(opt)
    elif args.sharding_stage > 0:
        from paddle2_amd.distributed.sharding import group_sharded_parallel

        level = {1: "os", 2: "os_g", 3: "p_g_os"}[args.sharding_stage]
        model, opt, _ = group_sharded_parallel(model, opt, level,
                                               group=fleet.get_hybrid_communicate_group().get_sharding_parallel_group())

    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    b, s = args.micro_batch, args.seq_len
    hcg = fleet.get_hybrid_communicate_group()
    # the data stream: one per data-parallel replica (dp x sharding ranks read different batches; the TP and PP
    # ranks of one replica read the same one)
    data_rank = hcg.get_data_parallel_rank() * sh + hcg.get_sharding_parallel_rank()
    gen = torch.Generator(device=dev).manual_seed(1000 + data_rank)
    # a fresh batch per step (pre-generated, outside the timed region); 8 x 4097 int64 = 262 KB each
    nb = args.warmup + args.steps
    if pp > 1:
        batches = [torch.randint(0, cfg.vocab_size, (b * acc, s + 1), generator=gen, device=dev) for _ in range(nb)]
    else:
        batches = [torch.randint(0, cfg.vocab_size, (b, s + 1), generator=gen, device=dev) for _ in range(nb * acc)]

    def step(i):
        if pp > 1:   # one pipelined step over acc micro-batches (1F1B), optimizer step and clear inside
            ids = paddle.Tensor._wrap(batches[i])
            return model.train_batch([ids[:, :-1], ids[:, 1:]], opt)
        for j in range(acc):
            ids = paddle.Tensor._wrap(batches[i * acc + j])
            loss = model(ids[:, :-1], labels=ids[:, 1:])
            (loss / acc if acc > 1 else loss).backward()
        opt.step()
        opt.clear_grad()
        return loss

    dbg = os.environ.get("PADDLE2_AMD_BENCH_DEBUG", "0") == "1"   # per-warmup-step sync + memory line (stderr)
    tw0 = time.perf_counter()
    for i in range(args.warmup):
        loss = step(i)
        if dbg and torch.cuda.is_available():
            torch.cuda.synchronize()
            extra = ""
            try:
                from paddle2_amd.device import allocator as _al

                if _al.is_active():
                    st = _al.stats(torch.cuda.current_device())
                    fr, tot = torch.cuda.mem_get_info()
                    extra = (f", device free {fr / 2**30:.1f} of {tot / 2**30:.1f} GiB"
                             f", reserved {st['reserved'] / 2**30:.1f} GiB, chunks {st['num_chunks']}, "
                             f"oom_retries {st['num_oom_retries']}, cross_stream {st['cross_stream_reuse']}, "
                             f"record_stream {st['record_stream']}, deferred {st['deferred_frees']}")
            except Exception as e:  # noqa: BLE001 - diagnostics only
                extra = f", allocator stats unavailable: {e}"
            print(f"[bench] warmup step {i} ok: allocated {torch.cuda.memory_allocated() / 2**30:.1f} GiB, "
                  f"peak {torch.cuda.max_memory_allocated() / 2**30:.1f} GiB{extra}", file=sys.stderr, flush=True)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    warm_step_s = (time.perf_counter() - tw0) / max(1, args.warmup)
    # bounded-time guard around the timed region (a hung collective must end the run, with a report, not stall it)
    import threading

    guard_s = args.hang_guard_s or max(300.0, 20.0 * warm_step_s * args.steps)
    guard = threading.Timer(guard_s, _hang_report, args=(guard_s,))
    guard.daemon = True
    guard.start()
    # communicator probe (outside the timed region, under the guard): bus bandwidth of the collectives sharding-3 runs
    probe = comm_probe(world, args.comm_probe_mb, torch.cuda.is_available())

    if world > 1:
        C.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        loss = step(args.warmup + i)
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    if world > 1:
        C.barrier()
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    elapsed = float(el.item())
    final_loss = float(loss)
    guard.cancel()
    peak = paddle.device.cuda.max_memory_allocated() / 2**30 if torch.cuda.is_available() else 0.0
    peaks = [round(peak, 1)]
    if world > 1:
        pt = torch.tensor([peak], dtype=torch.float64, device=dev)
        pl = [torch.zeros_like(pt) for _ in range(world)]
        torch.distributed.all_gather(pl, pt)
        peaks = [round(float(x.item()), 1) for x in pl]
    pgs = C.pg_status()
    comm_world = torch.distributed.get_world_size() if torch.distributed.is_initialized() else 1

    replicas = dp * sh   # data-parallel replicas: each trains its own b x acc sequences per step
    tokens = b * s * acc * args.steps * replicas
    tps = tokens / elapsed
    ms = elapsed / args.steps * 1000.0
    fpt = gpt_flops_per_token(cfg, s) if is_gpt else llama_flops_per_token(cfg, s)
    mfu = tps / world * fpt / 2.5e15
    if rank == 0:
        parts = ([f"mp{mp}" + ("+sp" if args.sp else "")] if mp > 1 else []) + \
            ([f"pp{pp}" + (f"v{vpp}" if vpp > 1 else "") + f"({args.pp_schedule if vpp == 1 else 'VPP'})"]
             if pp > 1 else []) + ([f"dp{dp}"] if dp > 1 else [])
        if sh > 1 or not parts:
            parts.append(f"sharding{args.sharding_stage}({sh})" if args.sharding_stage > 0
                         else f"single(no-sharding,debug)({sh})")
        par = "x".join(parts)
        if len(parts) == 1 and sh > 1 or (not (mp > 1 or pp > 1 or dp > 1) and args.sharding_stage > 0):
            par = f"sharding{args.sharding_stage}x{sh}"   # the headline's label (earlier rounds' records)
        names = {"llama2-7b": "Llama-2-7B", "llama2-13b": "Llama-2-13B", "gpt3-13b": "GPT-3 13B",
                 "gpt3-6.7b": "GPT-3 6.7B", "gpt3-1.3b": "GPT-3 1.3B", "tiny": "tiny-llama(debug)",
                 "gpt3-tiny": "tiny-gpt(debug)"}
        if args.model == "llama2-7b" and mp == pp == dp == 1 and args.sharding_stage == 3:
            metric = "tokens/sec (whole node) Llama-2-7B Fleet sharding-3 bf16"   # BASELINE.json's headline
        else:
            metric = f"tokens/sec (whole node) {names[args.model]} {'fp8' if args.fp8 else 'bf16'} {' x '.join(parts)}"
        out = {
            "metric": metric,
            "value": round(tps, 2),
            "unit": "tokens/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp8(e4m3/e5m2)+bf16" if (is_gpt and args.fp8) else "bf16",
            "data": "synthetic (fresh uniform random token ids per step), random-init weights",
            "config": {"model": args.model if not args.layers else f"{args.model}-L{args.layers}(debug)",
                       "global_batch": b * acc * replicas, "seq_len": s, "micro_batch_per_gpu": b,
                       "accumulate_steps": acc,
                       "parallelism": par, "layers": cfg.num_hidden_layers},
            "mfu_vs_2.5PF_dense": round(mfu, 4),
            "final_loss": round(final_loss, 4),
            "peak_mem_gb": round(peak, 1) if torch.cuda.is_available() else None,
            # self-diagnosis of the communicator that produced this number (a fallback would otherwise look valid)
            "pg_backend": pgs.get("backend"),
            "canary": pgs.get("canary"),
            "comm_world_size": comm_world,
            "ipc_allreduce": pgs.get("ipc"),
            "peak_mem_gb_per_rank": peaks,
            "stage3_keep_gathered": getattr(model, "keep_gathered", None),
            "hang_guard_s": round(guard_s, 1),
            "comm_probe": probe,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        # every rank is past its last collective before any tears down; then leave without running C++ static
        # destructors (a library thread still joinable there turns a finished run into SIGABRT at exit)
        C.barrier()
        C.destroy_process_group()
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)


if __name__ == "__main__":
    main()
