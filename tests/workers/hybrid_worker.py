"""Rank worker for hybrid-parallel tests (TP / PP / sharding-1 / DP via fleet) on gloo.

mode tp:   mp_degree=world; tiny Llama with TP layers trained 3 steps vs. a single-process model
           built from the gathered shards.
mode pp:   pp_degree=world; PipelineLayer MLP stack trained with 1F1B / FThenB / VPP vs. the same
           stack run single-process with gradient accumulation.
mode dpsh: dp=1, sharding_degree=world via fleet (DygraphShardingOptimizer) vs single process.
"""
import os
import sys

sys.path.insert(0, os.environ.get("PYTHONPATH", "."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import paddle2_amd as paddle  # noqa: E402
from paddle2_amd.distributed import fleet  # noqa: E402
from paddle2_amd.distributed import collective as C  # noqa: E402
from _dist import write_result  # noqa: E402

mode = sys.argv[1]
C.init_parallel_env()
rank, world = C.get_rank(), C.get_world_size()
steps = 3


def gather_full(t, axis, group):
    parts = [torch.empty_like(t) for _ in range(group.nranks)]
    dist.all_gather(parts, t.contiguous(), group=group.pg)
    return parts


def run_tp():
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": world, "pp_degree": 1}
    fleet.init(is_collective=True, strategy=strategy)
    hcg = fleet.get_hybrid_communicate_group()
    mpg = hcg.get_model_parallel_group()
    cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2,
                           tensor_parallel_degree=world)
    paddle.seed(3)
    m = LlamaForCausalLM(cfg)
    m = fleet.distributed_model(m)
    # gather the initial shards into a single-process state dict
    nh, nkv, d = cfg.num_attention_heads, cfg.num_key_value_heads, cfg.head_dim
    full = {}
    for name, p in m._layers.named_parameters():
        t = p._t.detach()
        if not getattr(p, "is_distributed", False):
            full[name] = t.clone()
            continue
        ax = p.split_axis
        parts = gather_full(t, ax, mpg)
        if "qkv_proj" in name:
            ql, kl = nh // world * d, nkv // world * d
            qs = [x[:, :ql] for x in parts]
            ks = [x[:, ql:ql + kl] for x in parts]
            vs = [x[:, ql + kl:] for x in parts]
            full[name] = torch.cat(qs + ks + vs, 1)
        elif "gate_up" in name:
            h = parts[0].shape[1] // 2
            full[name] = torch.cat([x[:, :h] for x in parts] + [x[:, h:] for x in parts], 1)
        else:
            full[name] = torch.cat(parts, ax)
    opt = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), weight_decay=0.01,
                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    opt = fleet.distributed_optimizer(opt)
    g = torch.Generator().manual_seed(5)
    data = [torch.randint(0, cfg.vocab_size, (2, 17), generator=g) for _ in range(steps)]
    losses = []
    for s in range(steps):
        ids = paddle.Tensor._wrap(data[s])
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    # reference
    cfg1 = LlamaConfig.tiny(dtype="float32", num_hidden_layers=2, num_attention_heads=4, num_key_value_heads=2)
    ref_m = LlamaForCausalLM(cfg1)
    ref_m.set_state_dict({k: paddle.Tensor._wrap(v) for k, v in full.items()})
    ref_o = paddle.optimizer.AdamW(1e-2, parameters=ref_m.parameters(), weight_decay=0.01,
                                   grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    ref = []
    for s in range(steps):
        ids = paddle.Tensor._wrap(data[s])
        loss = ref_m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        ref_o.step()
        ref_o.clear_grad()
        ref.append(float(loss))
    write_result({"losses": losses, "ref": ref})


class Blk(paddle.nn.Layer):
    def __init__(self, h):
        super().__init__()
        self.l1 = paddle.nn.Linear(h, 2 * h)
        self.l2 = paddle.nn.Linear(2 * h, h)

    def forward(self, x):
        return x + self.l2(paddle.nn.functional.gelu(self.l1(x)))


class Head(paddle.nn.Layer):
    def __init__(self, h, c):
        super().__init__()
        self.fc = paddle.nn.Linear(h, c)

    def forward(self, x):
        return self.fc(x)


def run_pp(schedule, vpp):
    from paddle2_amd.distributed.fleet.meta_parallel import LayerDesc, PipelineLayer

    M = 4
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": 1, "pp_degree": world}
    strategy.pipeline_configs = {"accumulate_steps": M, "micro_batch_size": 2}
    fleet.init(is_collective=True, strategy=strategy)
    H, Cn, L = 16, 5, 8
    loss_fn = lambda out, lab: paddle.nn.functional.cross_entropy(out, lab)  # noqa: E731
    descs = [LayerDesc(Blk, H) for _ in range(L)] + [LayerDesc(Head, H, Cn)]
    paddle.seed(11)
    # build the full stack once (same RNG order on every rank) to get reference weights
    ref_layers = [Blk(H) for _ in range(L)] + [Head(H, Cn)]
    ref_sd = [l.state_dict() for l in ref_layers]
    pl = PipelineLayer(descs, loss_fn=loss_fn, seg_method="uniform", num_virtual_pipeline_stages=vpp)
    # copy reference weights into the locally built pieces
    S = world
    for c, vs in enumerate(pl._chunk_vstages):
        lo = pl.segment_parts[vs]
        for i, item in enumerate(pl._model_chunks[c]._items):
            item.set_state_dict(ref_sd[lo + i])
    model = fleet.distributed_model(pl)
    if schedule == "FThenB":
        from paddle2_amd.distributed.fleet.meta_parallel import PipelineParallelFThenB

        model.__class__ = PipelineParallelFThenB
    if schedule == "ZBH1":
        from paddle2_amd.distributed.fleet.meta_parallel import PipelineParallelZeroBubble

        model.__class__ = PipelineParallelZeroBubble
    opt = paddle.optimizer.SGD(0.1, parameters=model.parameters())
    opt = fleet.distributed_optimizer(opt)
    g = torch.Generator().manual_seed(2)
    xs = [torch.randn(M * 2, 3, H, generator=g) for _ in range(steps)]
    ys = [torch.randint(0, Cn, (M * 2, 3), generator=g) for _ in range(steps)]
    losses = []
    for s in range(steps):
        loss = model.train_batch([paddle.Tensor._wrap(xs[s]), paddle.Tensor._wrap(ys[s])], opt)
        losses.append(float(loss))
    # reference: plain gradient accumulation
    seq = paddle.nn.Sequential(*ref_layers)
    ro = paddle.optimizer.SGD(0.1, parameters=seq.parameters())
    ref = []
    for s in range(steps):
        tot = 0.0
        for mb in range(M):
            x = paddle.Tensor._wrap(xs[s][mb * 2:(mb + 1) * 2])
            y = paddle.Tensor._wrap(ys[s][mb * 2:(mb + 1) * 2])
            l = loss_fn(seq(x), y) / M
            l.backward()
            tot += float(l)
        ro.step()
        ro.clear_grad()
        ref.append(tot)
    write_result({"losses": losses, "ref": ref})


def run_dpsh():
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": 1, "pp_degree": 1, "sharding_degree": world}
    fleet.init(is_collective=True, strategy=strategy)
    cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=2)

    def make():
        paddle.seed(7)
        m = LlamaForCausalLM(cfg)
        o = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), weight_decay=0.01,
                                   grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
        return m, o

    g = torch.Generator().manual_seed(99)
    data = [torch.randint(0, cfg.vocab_size, (world * 2, 33), generator=g) for _ in range(steps)]
    m, o = make()
    m = fleet.distributed_model(m)
    o = fleet.distributed_optimizer(o)
    losses = []
    for s in range(steps):
        ids = paddle.Tensor._wrap(data[s][rank * 2:(rank + 1) * 2])
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        o.step()
        o.clear_grad()
        t = loss._t.detach().clone()
        C._all_reduce_torch(t)
        losses.append(float(t) / world)
    csum = float(sum(p._t.double().sum() for p in m.parameters()))
    m2, o2 = make()
    ref = []
    for s in range(steps):
        ids = paddle.Tensor._wrap(data[s])
        loss = m2(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        o2.step()
        o2.clear_grad()
        ref.append(float(loss))
    csum_ref = float(sum(p._t.double().sum() for p in m2.parameters()))
    write_result({"losses": losses, "ref": ref, "csum": csum, "csum_ref": csum_ref})


def run_moe():
    from paddle2_amd.incubate.distributed.models.moe import MoELayer

    class E(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.l1 = paddle.nn.Linear(8, 16)
            self.l2 = paddle.nn.Linear(16, 8)

        def forward(self, x):
            return self.l2(paddle.nn.functional.gelu(self.l1(x)))

    group = C._get_default_group()
    paddle.seed(21)
    experts = [E() for _ in range(2 * world)]
    gate_ref = MoELayer(8, paddle.nn.LayerList(experts), gate={"type": "naive", "top_k": 2})
    local = paddle.nn.LayerList(experts[2 * rank:2 * rank + 2])
    moe = MoELayer(8, local, gate={"type": "naive", "top_k": 2}, moe_group=group)
    moe.gate.set_state_dict(gate_ref.gate.state_dict())
    g = torch.Generator().manual_seed(3)
    X = torch.randn(2 * world, 5, 8, generator=g)
    x = paddle.Tensor._wrap(X[2 * rank:2 * rank + 2].clone().requires_grad_(True))
    y = moe(x)
    (y * y).sum().backward()
    ep_grads = [p._t.grad.clone() for p in local.parameters()]
    for p in local.parameters():
        p.clear_gradient()
    xr = paddle.Tensor._wrap(X.clone().requires_grad_(True))
    yr = gate_ref(xr)
    (yr * yr).sum().backward()
    out_diff = float((y._t - yr._t[2 * rank:2 * rank + 2]).abs().max())
    xg_diff = float((x._t.grad - xr._t.grad[2 * rank:2 * rank + 2]).abs().max())
    eg = max(float((a - p._t.grad).abs().max()) for a, p in zip(ep_grads, local.parameters()))
    write_result({"out_diff": out_diff, "xg_diff": xg_diff, "eg": eg})


def run_pp_llama(mp):
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM, LlamaForCausalLMPipe

    pp = world // mp
    M = 2
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": mp, "pp_degree": pp}
    strategy.pipeline_configs = {"accumulate_steps": M, "micro_batch_size": 1,
                                 "enable_partial_send_recv": os.environ.get("PD_PARTIAL", "1") == "1"}
    fleet.init(is_collective=True, strategy=strategy)
    cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=4, tensor_parallel_degree=mp)
    g = torch.Generator().manual_seed(8)
    data = [torch.randint(0, cfg.vocab_size, (M, 17), generator=g) for _ in range(2)]
    paddle.seed(4)
    pipe = LlamaForCausalLMPipe(cfg)
    model = fleet.distributed_model(pipe)
    opt = fleet.distributed_optimizer(paddle.optimizer.SGD(0.5, parameters=model.parameters()))
    full = {}
    hcg = fleet.get_hybrid_communicate_group()
    mpg = hcg.get_model_parallel_group()

    def full_param(name, p):
        """gather a tensor-parallel shard over the mp group (concat along its split axis); fused per-rank
        [q_r|k_r|v_r] / [gate_r|up_r] column shards are re-assembled into the single-process layout"""
        t = p._t.detach().contiguous()
        if mp == 1 or not getattr(p, "is_distributed", False):
            return t.clone()
        parts = [torch.empty_like(t) for _ in range(mp)]
        torch.distributed.all_gather(parts, t, group=mpg.pg)
        if "qkv_proj" in name:
            d = cfg.head_dim
            nh, nkv = cfg.num_attention_heads // mp, cfg.num_key_value_heads // mp
            qs = [x[:, :nh * d] for x in parts]
            ks = [x[:, nh * d:(nh + nkv) * d] for x in parts]
            vs = [x[:, (nh + nkv) * d:] for x in parts]
            return torch.cat(qs + ks + vs, dim=1)
        if "gate_up_fused_proj" in name:
            f = t.shape[1] // 2
            return torch.cat([x[:, :f] for x in parts] + [x[:, f:] for x in parts], dim=1)
        return torch.cat(parts, dim=p.split_axis)

    if True:
        # single-process reference with the same weights (pipe param names -> LlamaForCausalLM names)
        for c, vs in enumerate(pipe._chunk_vstages):
            lo = pipe.segment_parts[vs]
            for i, item in enumerate(pipe._model_chunks[c]._items):
                idx = lo + i
                for k, p in item.named_parameters():
                    v = paddle.Tensor._wrap(full_param(k, p))
                    if idx == 0:
                        name = "llama." + k
                    elif idx <= cfg.num_hidden_layers:
                        name = f"llama.layers.{idx - 1}." + k
                    elif idx == cfg.num_hidden_layers + 1:
                        name = "llama." + k
                    else:
                        name = "lm_head." + k
                    full[name] = v._t.detach().clone()
    losses = []
    for ids in data:
        ids = paddle.Tensor._wrap(ids)
        losses.append(float(model.train_batch([ids[:, :-1], ids[:, 1:]], opt)))
    out = {"losses": losses}
    if True:
        objs = [None] * world
        torch.distributed.all_gather_object(objs, {k: v.numpy() for k, v in full.items()})
        merged = {}
        for o in objs:
            merged.update(o)
        ref = LlamaForCausalLM(LlamaConfig.tiny(dtype="float32", num_hidden_layers=4))
        ref.set_state_dict({k: paddle.to_tensor(v) for k, v in merged.items()})
        ro = paddle.optimizer.SGD(0.5, parameters=ref.parameters())
        rl = []
        for ids in data:
            tot = 0.0
            for mb in range(M):
                x = paddle.Tensor._wrap(ids[mb:mb + 1])
                l = ref(x[:, :-1], labels=x[:, 1:]) / M
                l.backward()
                tot += float(l)
            ro.step()
            ro.clear_grad()
            rl.append(tot)
        out["ref"] = rl
    write_result(out)


def run_gpt_sp():
    from paddle2_amd.models import GPTConfig, GPTForCausalLM

    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": world, "pp_degree": 1}
    fleet.init(is_collective=True, strategy=strategy)
    g = torch.Generator().manual_seed(6)
    data = [torch.randint(0, 512, (2, 33), generator=g) for _ in range(3)]

    def run(sp, init_sd=None):
        paddle.seed(9)
        m = GPTForCausalLM(GPTConfig.tiny(dtype="float32", tensor_parallel_degree=world, sequence_parallel=sp))
        if init_sd is not None:
            m.set_state_dict(init_sd)
        sd0 = {k: paddle.Tensor._wrap(v._t.detach().clone()) for k, v in m.state_dict().items()}
        model = fleet.distributed_model(m)
        opt = fleet.distributed_optimizer(paddle.optimizer.AdamW(1e-2, parameters=model.parameters(),
                                                                 grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0)))
        out = []
        for ids in data:
            ids = paddle.Tensor._wrap(ids)
            loss = model(ids[:, :-1], labels=ids[:, 1:])
            loss.backward()
            opt.step()
            opt.clear_grad()
            out.append(float(loss))
        return out, sd0

    ref, sd0 = run(False)
    sp, _ = run(True, sd0)
    write_result({"losses": sp, "ref": ref})


def run_gpt_fp8_hybrid(kind):
    """BASELINE config 5 in miniature: GPT fp8 linears with TP 2 (+ SP) inside, on 4 ranks.
    kind sh3: TP2 + SP + group-sharded stage 3 over the other 2 ranks (bench.py --mp 2 --sp, sharding 2);
    kind dp:  TP2 (no SP) + 2-way data parallel through the fleet wrappers — the reference configuration.
    Same init (model-parallel RNG per mp rank), same global batch of 4 sequences per step (2 per replica), global-norm
    clipping on: the mean losses must agree."""
    from paddle2_amd.models import GPTConfig, GPTForCausalLM

    sp = kind == "sh3"
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1 if sp else 2, "mp_degree": 2, "pp_degree": 1,
                               "sharding_degree": 2 if sp else 1}
    fleet.init(is_collective=True, strategy=strategy)
    hcg = fleet.get_hybrid_communicate_group()
    g = torch.Generator().manual_seed(6)
    data = [torch.randint(0, 512, (4, 33), generator=g) for _ in range(4)]
    paddle.seed(9)
    m = GPTForCausalLM(GPTConfig.tiny(dtype="float32", tensor_parallel_degree=2, sequence_parallel=sp,
                                      use_fp8=True))
    opt = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), grad_clip=paddle.nn.ClipGradByGlobalNorm(0.5))
    if sp:
        from paddle2_amd.distributed.sharding import group_sharded_parallel

        m, opt, _ = group_sharded_parallel(m, opt, "p_g_os", group=hcg.get_sharding_parallel_group())
        rep = hcg.get_sharding_parallel_rank()
    else:
        m = fleet.distributed_model(m)
        opt = fleet.distributed_optimizer(opt)
        rep = hcg.get_data_parallel_rank()
    out = []
    for ids in data:
        ids = paddle.Tensor._wrap(ids[2 * rep:2 * rep + 2])
        loss = m(ids[:, :-1], labels=ids[:, 1:])
        loss.backward()
        opt.step()
        opt.clear_grad()
        t = loss._t.detach().float().clone()
        dist.all_reduce(t)
        out.append(float(t) / world)
    write_result({"losses": out})


def _llama_ref_run(cfg, data, k, make):
    """single process: every step accumulates k micro-batches of the GLOBAL batch (loss / k)"""
    m, o = make()
    ref = []
    for s in range(len(data)):
        tot = 0.0
        for j in range(k):
            ids = paddle.Tensor._wrap(data[s][j])
            loss = m(ids[:, :-1], labels=ids[:, 1:]) / k
            loss.backward()
            tot += float(loss)
        o.step()
        o.clear_grad()
        ref.append(tot)
    return ref, m


def run_shv2(variant):
    """Sharding V2 (split_param) / dp gradient-hook overlap vs. a single process (4 ranks).
    v2:     sharding 4, split_param, 64 KiB buckets (parameters split across ranks), reduce at step
    v2ov:   + comm_overlap (reduce-scatter from gradient hooks) and gradient merge k=2
    dp2sh2: dp 2 x sharding 2, split_param + comm_overlap (owned shards all-reduced over dp)
    dpgm:   dp 4 (DataParallel reducer only), gradient merge k=2
    v1:     sharding 4, V1 (whole-parameter ownership) — the V2 == V1 anchor"""
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    dp = {"v2": 1, "v2ov": 1, "dp2sh2": 2, "dpgm": 4, "v1": 1}[variant]
    sh = world // dp
    k = 2 if variant in ("v2ov", "dpgm") else 1
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {
        "dp_degree": dp, "mp_degree": 1, "pp_degree": 1, "sharding_degree": sh,
        "sharding_configs": {"split_param": variant != "v1", "comm_buffer_size_MB": 1,
                             "comm_overlap": variant in ("v2ov", "dp2sh2")},
        "pp_configs": {"dp_comm_overlap": variant == "dpgm"}}   # ignored without pp: the reducer overlaps
    if k > 1:
        strategy.gradient_merge = True
        strategy.gradient_merge_configs = {"k_steps": k, "avg": True}
    fleet.init(is_collective=True, strategy=strategy)
    cfg = LlamaConfig.tiny(dtype="float32", num_hidden_layers=2)

    def make():
        paddle.seed(7)
        m = LlamaForCausalLM(cfg)
        o = paddle.optimizer.AdamW(1e-2, parameters=m.parameters(), weight_decay=0.01,
                                   grad_clip=paddle.nn.ClipGradByGlobalNorm(1.0))
        return m, o

    g = torch.Generator().manual_seed(99)
    # data[s][j]: global micro-batch j of step s; rank r (data-parallel index over dp x sharding) takes rows 2r:2r+2
    data = [[torch.randint(0, cfg.vocab_size, (world * 2, 33), generator=g) for _ in range(k)] for _ in range(steps)]
    m, o = make()
    m = fleet.distributed_model(m)
    o = fleet.distributed_optimizer(o)
    from paddle2_amd.distributed.fleet.meta_optimizers.dygraph_optimizer.hybrid_parallel_optimizer import \
        DygraphShardingOptimizerV2
    info = {"v2": isinstance(o._inner_opt, DygraphShardingOptimizerV2),
            "buckets": len(getattr(o._inner_opt, "_buffers", [])) or len(o._dp_buffers)}
    losses = []
    for s in range(steps):
        tot = 0.0
        for j in range(k):
            ids = paddle.Tensor._wrap(data[s][j][rank * 2:(rank + 1) * 2])
            loss = m(ids[:, :-1], labels=ids[:, 1:])
            loss.backward()
            o.step()
            o.clear_grad()
            t = loss._t.detach().clone()
            C._all_reduce_torch(t)
            tot += float(t) / world / k
        losses.append(tot)
    csum = float(sum(p._t.double().sum() for p in m.parameters()))
    ref, m2 = _llama_ref_run(cfg, data, k, make)
    csum_ref = float(sum(p._t.double().sum() for p in m2.parameters()))
    write_result({"losses": losses, "ref": ref, "csum": csum, "csum_ref": csum_ref, **info})


def run_pp_hybrid(kind):
    """pp 2 x (dp 2 with dp_comm_overlap | sharding 2 V2 with sharding_comm_overlap): the pipeline's per-micro-batch
    backward fires the gradient hooks; communication happens after the last micro-batch == grad accumulation"""
    from paddle2_amd.distributed.fleet.meta_parallel import LayerDesc, PipelineLayer

    M, MB = 4, 2
    strategy = fleet.DistributedStrategy()
    hc = {"dp_degree": 1, "mp_degree": 1, "pp_degree": 2, "sharding_degree": 1,
          "pp_configs": {"dp_comm_overlap": kind in ("dp", "dly"), "sharding_comm_overlap": kind == "sh",
                         "delay_scale_loss": kind == "dly"}}
    if kind in ("dp", "dly"):
        hc["dp_degree"] = 2
    else:
        hc["sharding_degree"] = 2
        hc["sharding_configs"] = {"split_param": True, "comm_buffer_size_MB": 1}
    strategy.hybrid_configs = hc
    strategy.pipeline_configs = {"accumulate_steps": M, "micro_batch_size": MB}
    fleet.init(is_collective=True, strategy=strategy)
    hcg = fleet.get_hybrid_communicate_group()
    didx = hcg.get_data_parallel_rank() if kind in ("dp", "dly") else hcg.get_sharding_parallel_rank()
    H, Cn, L = 16, 5, 4
    loss_fn = lambda out, lab: paddle.nn.functional.cross_entropy(out, lab)  # noqa: E731
    descs = [LayerDesc(Blk, H) for _ in range(L)] + [LayerDesc(Head, H, Cn)]
    paddle.seed(11)
    ref_layers = [Blk(H) for _ in range(L)] + [Head(H, Cn)]
    ref_sd = [l.state_dict() for l in ref_layers]
    pl = PipelineLayer(descs, loss_fn=loss_fn, seg_method="uniform")
    for c, vs in enumerate(pl._chunk_vstages):
        lo = pl.segment_parts[vs]
        for i, item in enumerate(pl._model_chunks[c]._items):
            item.set_state_dict(ref_sd[lo + i])
    model = fleet.distributed_model(pl)
    opt = fleet.distributed_optimizer(paddle.optimizer.AdamW(0.05, parameters=model.parameters()))
    g = torch.Generator().manual_seed(2)
    D = 2
    xs = [torch.randn(D * M * MB, 3, H, generator=g) for _ in range(steps)]
    ys = [torch.randint(0, Cn, (D * M * MB, 3), generator=g) for _ in range(steps)]
    lo, hi = didx * M * MB, (didx + 1) * M * MB
    losses = []
    for s in range(steps):
        loss = model.train_batch([paddle.Tensor._wrap(xs[s][lo:hi]), paddle.Tensor._wrap(ys[s][lo:hi])], opt)
        t = loss._t.detach().clone().reshape(1)
        C._all_reduce_torch(t)
        losses.append(float(t) / world)
    seq = paddle.nn.Sequential(*ref_layers)
    ro = paddle.optimizer.AdamW(0.05, parameters=seq.parameters())
    ref = []
    for s in range(steps):
        tot = 0.0
        for mb in range(D * M):
            x = paddle.Tensor._wrap(xs[s][mb * MB:(mb + 1) * MB])
            y = paddle.Tensor._wrap(ys[s][mb * MB:(mb + 1) * MB])
            l = loss_fn(seq(x), y) / (D * M)
            l.backward()
            tot += float(l)
        ro.step()
        ro.clear_grad()
        ref.append(tot)
    write_result({"losses": losses, "ref": ref})


def run_mpsync(sync_mode):
    """mp_configs sync_grad / sync_param / sync_moment (+ sync_mode) on a replicated parameter whose gradient
    differs per mp rank, and need_broadcast_data (inputs replaced by mp rank 0's)."""
    strategy = fleet.DistributedStrategy()
    strategy.hybrid_configs = {"dp_degree": 1, "mp_degree": world, "pp_degree": 1,
                               "mp_configs": {"sync_grad": True, "sync_param": True, "sync_moment": True,
                                              "sync_mode": sync_mode, "need_broadcast_data": False}}
    strategy.sync_param_name = ["layer_norm"]
    fleet.init(is_collective=True, strategy=strategy)

    class M(paddle.nn.Layer):
        def __init__(self):
            super().__init__()
            self.w = paddle.create_parameter([8], "float32", name="layer_norm_0.w_0")
            self.u = paddle.create_parameter([8], "float32", name="other_0.w_0")   # not in sync_param_name

        def forward(self, x):
            return ((x * self.w).sum() ** 2 + (x * self.u).sum() ** 2)

    paddle.seed(1)
    m = M()
    model = fleet.distributed_model(m)
    opt = fleet.distributed_optimizer(paddle.optimizer.AdamW(0.1, parameters=model.parameters()))
    xs = [torch.randn(world, 8, generator=torch.Generator().manual_seed(s)) for s in range(2)]
    for x in xs:
        loss = model(paddle.Tensor._wrap(x[rank].clone()))
        loss.backward()
        opt.step()
        opt.clear_grad()
    w = m.w._t.detach().clone()
    u = m.u._t.detach().clone()
    m1 = opt._base_opt._accumulators["moment1"][m.w.name].clone()
    ws = [torch.empty_like(w) for _ in range(world)]
    us = [torch.empty_like(u) for _ in range(world)]
    ms = [torch.empty_like(m1) for _ in range(world)]
    dist.all_gather(ws, w)
    dist.all_gather(us, u)
    dist.all_gather(ms, m1)
    out = {"w_equal": all(torch.equal(ws[0], t) for t in ws), "m_equal": all(torch.equal(ms[0], t) for t in ms),
           "u_differ": not all(torch.equal(us[0], t) for t in us)}
    if sync_mode == "average":
        # single process: the replicated param sees the mp-averaged gradient
        paddle.seed(1)
        r = M()
        ro = paddle.optimizer.AdamW(0.1, parameters=[r.w])
        for x in xs:
            loss = sum(((x[k] * r.w._t).sum() ** 2) for k in range(world)) / world
            loss.backward()
            ro.step()
            ro.clear_grad()
        out["w_ref_diff"] = float((r.w._t.detach() - w).abs().max())
    # need_broadcast_data: a TensorParallel forward sees mp rank 0's input
    model._need_broadcast_data = True
    x = torch.full((8,), float(rank + 1))
    model(paddle.Tensor._wrap(x))
    out["bcast_input"] = float(x[0])
    write_result(out)


if mode == "tp":
    run_tp()
elif mode == "pp":
    run_pp(sys.argv[2], int(sys.argv[3]))
elif mode == "dpsh":
    run_dpsh()
elif mode == "moe":
    run_moe()
elif mode == "gpt_sp":
    run_gpt_sp()
elif mode == "gpt_fp8_hybrid":
    run_gpt_fp8_hybrid(sys.argv[2])
elif mode == "shv2":
    run_shv2(sys.argv[2])
elif mode == "mpsync":
    run_mpsync(sys.argv[2])
elif mode == "pp_hybrid":
    run_pp_hybrid(sys.argv[2])
elif mode == "pp_llama":
    run_pp_llama(int(sys.argv[2]))
