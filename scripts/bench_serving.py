"""Serving benchmark: Llama-2-7B decode throughput on one MI355X (paged KV cache, flash-decoding
kernel, HIP-graph decode step).  Random-init weights, synthetic prompts."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.models import LlamaConfig, LlamaForCausalLM  # noqa: E402
from paddle2_amd.serving.generation import LlamaGenerator  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=64)
ap.add_argument("--prompt", type=int, default=1024)
ap.add_argument("--new", type=int, default=64)
ap.add_argument("--no-graph", action="store_true")
ap.add_argument("--layers", type=int, default=None)
ap.add_argument("--prefill", default="batch", choices=["batch", "seq"],
                help="prefill all prompts as one packed batch (default) or one at a time")
ap.add_argument("--gemm-autotune", default="auto", choices=["auto", "tune", "off"],
                help="hipBLASLt selection cache (tuning/gemm_gfx950.csv) for the GEMMs that route to hipBLASLt (the "
                     "wide b64 decode projections): auto = use it if present; tune = search and extend it (eager "
                     "steps only: TunableOp does not tune inside a HIP-graph capture, use with --no-graph)")
args = ap.parse_args()

if args.gemm_autotune != "off":
    from paddle2_amd.incubate import autotune

    if args.gemm_autotune == "tune" or os.path.exists(autotune.DEFAULT_GEMM_CACHE):
        autotune.enable_gemm_autotune(tuning=args.gemm_autotune == "tune")

paddle.set_device("gpu:0")
paddle.seed(0)
cfg = LlamaConfig.llama2_7b()
if args.layers:
    cfg.num_hidden_layers = args.layers
with torch.device("cuda"):
    model = LlamaForCausalLM(cfg)
model.eval()
gen = LlamaGenerator(model, max_batch=args.batch, max_seq_len=args.prompt + args.new + 16, block_size=64,
                     use_graph=not args.no_graph)
g = torch.Generator().manual_seed(0)
prompts = [torch.randint(0, cfg.vocab_size, (args.prompt,), generator=g) for _ in range(args.batch)]
B = args.batch
slots = list(range(B))
if args.prefill == "batch":
    # one untimed packed prefill (kernel routes, workspaces), then the timed one
    gen.prefill_batch(slots, prompts)
    for i in slots:
        gen.cache.free(i)
torch.cuda.synchronize()
t0 = time.perf_counter()
if args.prefill == "batch":   # all prompts as one packed token batch (varlen attention)
    first = gen.prefill_batch(slots, prompts).argmax(-1).tolist()
else:                         # one prompt at a time
    first = [int(gen.prefill(i, p).argmax()) for i, p in enumerate(prompts)]
torch.cuda.synchronize()
t_prefill = time.perf_counter() - t0
for i in slots:
    gen.cache.allocate(i, args.prompt + args.new + 1)
toks = torch.tensor(first, device="cuda")
pos = torch.full((B,), args.prompt, dtype=torch.int32, device="cuda")
for _ in range(3):  # capture + warm
    logits = gen.decode_step(toks, pos)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(args.new):
    logits = gen.decode_step(toks, pos)
    toks = logits.argmax(-1)
    pos = pos + 1
torch.cuda.synchronize()
t_dec = time.perf_counter() - t0
print(json.dumps({"metric": "Llama-2-7B decode tokens/s (1x MI355X)", "batch": B, "prompt_len": args.prompt,
                  "new_tokens": args.new, "hip_graph": not args.no_graph, "layers": cfg.num_hidden_layers,
                  "prefill": args.prefill, "prefill_tokens_per_s": round(B * args.prompt / t_prefill, 1),
                  "decode_tokens_per_s": round(B * args.new / t_dec, 1),
                  "decode_ms_per_step": round(t_dec / args.new * 1000, 3)}), flush=True)
