"""Long-tail ops of the reference inventory that have no same-named public function (reference
paddle/phi/ops/yaml/ops.yaml, fused_ops.yaml, sparse_ops.yaml; kernels under paddle/phi/kernels/ named per op).

Functional optimizer steps (``nadam_``, ``radam_``, ``asgd_``, ``rprop_``, ``decayed_adagrad``, ``ftrl``,
``dpsgd``, ``lars_momentum_``, ``average_accumulates_``) update their tensors in place like the reference's
inplace kernels; MoE routing helpers (``number_count``, ``assign_pos``, ``limit_by_capacity``,
``prune_gate_by_capacity``, ``random_routing``) follow python/paddle/distributed/models/moe/utils.py; the fused
inference ops compose the framework's native kernels (layer_norm / linear / activations).  Registered through
``op_schema.ALIASES`` so ``_C_ops.<name>`` resolves them.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from .op_schema import _lr, _raw, _upd, _wrap


def _p(param, master_param, multi_precision):
    return _raw(master_param if (multi_precision and master_param is not None) else param).float()


def _store(param, master_param, multi_precision, new):
    _upd(param, new)
    if master_param is not None and multi_precision:
        _upd(master_param, new)


# ------------------------------------------------------------------------------------------ optimizers
@torch.no_grad()
def nadam_(param, grad, learning_rate, momentum_decay_pow, beta2_pow, mu_product, moment1, moment2,
           master_param=None, beta1=0.9, beta2=0.999, epsilon=1e-8, momentum_decay=0.004, multi_precision=False):
    """phi nadam kernel: momentum_decay_pow carries 0.96^t, mu_product the running product of mu_t."""
    p, g = _p(param, master_param, multi_precision), _raw(grad).float()
    mdp = _raw(momentum_decay_pow).float() * 0.96
    mu_t = beta1 * (1 - 0.5 * mdp ** momentum_decay)
    mu_t1 = beta1 * (1 - 0.5 * (mdp * 0.96) ** momentum_decay)
    mup = _raw(mu_product).float() * mu_t
    b2p = _raw(beta2_pow).float() * beta2
    m1 = _raw(moment1).float() * beta1 + (1 - beta1) * g
    m2 = _raw(moment2).float() * beta2 + (1 - beta2) * g * g
    m1h = mu_t1 * m1 / (1 - mup * mu_t1) + (1 - mu_t) * g / (1 - mup)
    m2h = m2 / (1 - b2p)
    _store(param, master_param, multi_precision, p - _lr(learning_rate) * m1h / (m2h.sqrt() + epsilon))
    for dst, v in ((momentum_decay_pow, mdp), (mu_product, mup), (beta2_pow, b2p), (moment1, m1), (moment2, m2)):
        _upd(dst, v)
    return param, momentum_decay_pow, beta2_pow, mu_product, moment1, moment2, master_param


@torch.no_grad()
def radam_(param, grad, learning_rate, beta1_pow, beta2_pow, rho, moment1, moment2, master_param=None, beta1=0.9,
           beta2=0.999, epsilon=1e-8, multi_precision=False):
    """phi radam kernel: beta pows advance first, rho carries the step count t (as a float)."""
    p, g = _p(param, master_param, multi_precision), _raw(grad).float()
    b1p = _raw(beta1_pow).float() * beta1
    b2p = _raw(beta2_pow).float() * beta2
    t = _raw(rho).float() + 1
    rho_inf = 2 / (1 - beta2) - 1
    rho_t = rho_inf - 2 * t * b2p / (1 - b2p)
    m1 = _raw(moment1).float() * beta1 + (1 - beta1) * g
    m2 = _raw(moment2).float() * beta2 + (1 - beta2) * g * g
    mh = m1 / (1 - b1p)
    r = torch.sqrt(((rho_t - 4) * (rho_t - 2) * rho_inf / ((rho_inf - 4) * (rho_inf - 2) * rho_t)).clamp(min=0))
    adapt = r * mh * torch.sqrt(1 - b2p) / (m2.sqrt() + epsilon)
    upd = torch.where(rho_t > 5, adapt, mh)
    _store(param, master_param, multi_precision, p - _lr(learning_rate) * upd)
    for dst, v in ((beta1_pow, b1p), (beta2_pow, b2p), (rho, t), (moment1, m1), (moment2, m2)):
        _upd(dst, v)
    return param, beta1_pow, beta2_pow, rho, moment1, moment2, master_param


@torch.no_grad()
def asgd_(param, grad, learning_rate, d, y, n, master_param=None, multi_precision=False):
    """phi asgd kernel: d = d - y + g; y = g; p -= lr / n * d (n = min(step, batch_num), supplied)."""
    p, g = _p(param, master_param, multi_precision), _raw(grad).float()
    dn = _raw(d).float() - _raw(y).float() + g
    _store(param, master_param, multi_precision, p - _lr(learning_rate) / _raw(n).float().reshape(-1)[0] * dn)
    _upd(d, dn)
    _upd(y, g)
    return param, d, y, master_param


@torch.no_grad()
def rprop_(param, grad, prev, learning_rate, master_param=None, learning_rate_range=(1e-5, 50), etas=(0.5, 1.2),
           multi_precision=False):
    """phi rprop kernel: per-element step sizes (learning_rate is a tensor like param)."""
    p, g = _p(param, master_param, multi_precision), _raw(grad).float()

    def pair(v):
        r = _raw(v)
        return [float(a) for a in (r.reshape(-1).tolist() if isinstance(r, torch.Tensor) else v)]

    lo, hi = pair(learning_rate_range)
    em, ep = pair(etas)
    s = g * _raw(prev).float()
    lrs = _raw(learning_rate).float()
    lrs = torch.where(s > 0, lrs * ep, torch.where(s < 0, lrs * em, lrs)).clamp(lo, hi)
    g = torch.where(s < 0, torch.zeros_like(g), g)
    _store(param, master_param, multi_precision, p - torch.sign(g) * lrs)
    _upd(prev, g)
    _upd(learning_rate, lrs)
    return param, prev, learning_rate, master_param


@torch.no_grad()
def decayed_adagrad(param, grad, moment, learning_rate, decay=0.95, epsilon=1e-6):
    g = _raw(grad).float()
    m = _raw(moment).float() * decay + (1 - decay) * g * g
    _upd(param, _raw(param).float() - _lr(learning_rate) * g / (m.sqrt() + epsilon))
    _upd(moment, m)
    return param, moment


@torch.no_grad()
def ftrl(param, squared_accumulator, linear_accumulator, grad, learning_rate, l1=0.0, l2=0.0, lr_power=-0.5):
    """FTRL-proximal (phi ftrl kernel): returns (param, squared_accum, linear_accum) updated in place."""
    p, g = _raw(param).float(), _raw(grad).float()
    n, z = _raw(squared_accumulator).float(), _raw(linear_accumulator).float()
    lr = _lr(learning_rate)
    nn_ = n + g * g
    if lr_power == -0.5:
        sigma = (nn_.sqrt() - n.sqrt()) / lr
        denom = nn_.sqrt() / lr + 2 * l2
    else:
        sigma = (nn_.pow(-lr_power) - n.pow(-lr_power)) / lr
        denom = nn_.pow(-lr_power) / lr + 2 * l2
    z = z + g - sigma * p
    newp = torch.where(z.abs() > l1, (torch.sign(z) * l1 - z) / denom, torch.zeros_like(z))
    _upd(param, newp)
    _upd(squared_accumulator, nn_)
    _upd(linear_accumulator, z)
    return param, squared_accumulator, linear_accumulator


@torch.no_grad()
def dpsgd(param, grad, learning_rate, clip=10.0, batch_size=16.0, sigma=1.0, seed=0):
    """Differentially private SGD (phi dpsgd kernel): clip the gradient to L2 norm ``clip``, add Gaussian noise
    of std ``sigma * clip`` scaled by 1 / batch_size, then an SGD step."""
    g = _raw(grad).float()
    norm = g.norm()
    g = g / torch.clamp(norm / clip, min=1.0)
    gen = torch.Generator(device=g.device)
    gen.manual_seed(int(seed))
    noise = torch.randn(g.shape, generator=gen, device=g.device) * (sigma * clip)
    g = g + noise / batch_size
    _upd(param, _raw(param).float() - _lr(learning_rate) * g)
    return param


@torch.no_grad()
def lars_momentum_(param, grad, velocity, learning_rate, master_param=None, mu=0.9, lars_coeff=0.001,
                   lars_weight_decay=(0.0005,), epsilon=0.0, multi_precision=False, rescale_grad=1.0):
    """LARS momentum for one (or a list of) parameter(s) (phi lars_momentum kernel)."""
    many = isinstance(param, (list, tuple))
    ps, gs, vs = (param, grad, velocity) if many else ([param], [grad], [velocity])
    lrs = learning_rate if isinstance(learning_rate, (list, tuple)) else [learning_rate] * len(ps)
    mps = master_param if isinstance(master_param, (list, tuple)) else [master_param] * len(ps)
    wds = list(lars_weight_decay) if isinstance(lars_weight_decay, (list, tuple)) else [lars_weight_decay]
    for i, (pp, gg, vv) in enumerate(zip(ps, gs, vs)):
        wd = wds[i] if i < len(wds) else wds[-1]
        p, g = _p(pp, mps[i], multi_precision), _raw(gg).float() * rescale_grad
        pn, gn = p.norm(), g.norm()
        local = torch.where((pn > 0) & (gn > 0), lars_coeff * pn / (gn + wd * pn + epsilon), torch.ones_like(pn))
        v = _raw(vv).float() * mu + _lr(lrs[i]) * local * (g + wd * p)
        _store(pp, mps[i], multi_precision, p - v)
        _upd(vv, v)
    return param, velocity, master_param


@torch.no_grad()
def average_accumulates_(param, in_sum_1, in_sum_2, in_sum_3, in_num_accumulates, in_old_num_accumulates,
                         in_num_updates, average_window=0.0, max_average_window=10000, min_average_window=10000):
    """ModelAverage accumulation (phi average_accumulates kernel): sum_1 += param; every 16384 updates sum_1 is
    folded into sum_2; when the window is full, sums roll into sum_3 and restart."""
    p = _raw(param).float()
    s1, s2, s3 = (_raw(x).float() for x in (in_sum_1, in_sum_2, in_sum_3))
    na = int(_raw(in_num_accumulates).reshape(-1)[0]) + 1
    ona = int(_raw(in_old_num_accumulates).reshape(-1)[0])
    nu = int(_raw(in_num_updates).reshape(-1)[0]) + 1
    s1 = s1 + p
    if nu % 16384 == 0:
        s2, s1 = s2 + s1, torch.zeros_like(s1)
    if na >= min_average_window and na >= min(max_average_window, nu * average_window):
        s3, s1, s2 = s1 + s2, torch.zeros_like(s1), torch.zeros_like(s2)
        ona, na = na, 0
    for dst, v in ((in_sum_1, s1), (in_sum_2, s2), (in_sum_3, s3)):
        _upd(dst, v)
    for dst, v in ((in_num_accumulates, na), (in_old_num_accumulates, ona), (in_num_updates, nu)):
        _raw(dst).fill_(v)
    return in_sum_1, in_sum_2, in_sum_3, in_num_accumulates, in_old_num_accumulates, in_num_updates


# ------------------------------------------------------------------------------------------ MoE routing
def number_count(numbers, upper_range):
    """Count of each expert id in ``numbers`` (ids < 0 are dropped)."""
    n = _raw(numbers).reshape(-1).long()
    n = n[(n >= 0) & (n < upper_range)]
    return _wrap(torch.bincount(n, minlength=upper_range).to(torch.int64))


def assign_pos(x, cum_count, eff_num_len):
    """Token positions grouped by expert: out[cum_count[e-1] .. cum_count[e]) lists the tokens routed to e."""
    ids = _raw(x).reshape(-1).long()
    valid = ids >= 0
    order = torch.argsort(torch.where(valid, ids, torch.full_like(ids, 1 << 40)), stable=True)
    n = int(_raw(eff_num_len).reshape(-1)[0]) if isinstance(_raw(eff_num_len), torch.Tensor) else int(eff_num_len)
    return _wrap(order[:n].to(torch.int64))


def limit_by_capacity(expert_count, capacity, n_worker):
    """Clip per-(worker, expert) counts so each expert's total over workers stays within its capacity, filling
    workers in order (moe utils _limit_by_capacity)."""
    ec = _raw(expert_count).reshape(int(n_worker), -1).long()
    cap = _raw(capacity).reshape(-1).long().clone()
    out = torch.zeros_like(ec)
    for w in range(ec.shape[0]):
        take = torch.minimum(ec[w], cap)
        out[w] = take
        cap -= take
    return _wrap(out.reshape(-1))


def prune_gate_by_capacity(gate_idx, expert_count, n_expert, n_worker):
    """Tokens beyond their expert's remaining count get gate -1 (dropped), in token order: a token is kept iff its
    rank among the earlier tokens routed to the same expert is below that expert's count (vectorised: stable sort by
    expert, rank = position - first position of the expert's run; no per-token host loop)."""
    g = _raw(gate_idx)
    gi = g.reshape(-1).long()
    cnt = _raw(expert_count).reshape(-1).long().to(gi.device)
    ne = cnt.numel()
    valid = (gi >= 0) & (gi < ne)
    key = torch.where(valid, gi, torch.full_like(gi, ne))
    order = torch.argsort(key, stable=True)
    sk = key[order]
    rank_sorted = torch.arange(sk.numel(), device=gi.device) - torch.searchsorted(sk, sk, right=False)
    rank = torch.empty_like(rank_sorted)
    rank[order] = rank_sorted
    cap = torch.cat([cnt, cnt.new_zeros(1)])[key]
    out = torch.where(valid & (rank < cap), gi, torch.full_like(gi, -1))
    return _wrap(out.to(g.dtype).reshape(g.shape))


def random_routing(topk_idx, topk_value, prob):
    """GShard random routing: the 2nd expert is kept only where 2 * value >= prob (uniform sample)."""
    idx = _raw(topk_idx).clone()
    v = _raw(topk_value)
    p = _raw(prob).reshape(-1)
    drop = 2 * v[:, 1] < p[: idx.shape[0]]
    idx[:, 1] = torch.where(drop, torch.full_like(idx[:, 1], -1), idx[:, 1])
    return _wrap(idx)


# ------------------------------------------------------------------------------------------ misc tensor ops
def partial_concat(x, start_index=0, length=-1):
    """Concatenate columns [start, start+length) of every 2-D input along axis 1."""
    outs = []
    for t in x:
        r = _raw(t)
        s = start_index % r.shape[1] if start_index < 0 else start_index
        e = r.shape[1] if length < 0 else s + length
        outs.append(r[:, s:e])
    return _wrap(torch.cat(outs, dim=1))


def partial_sum(x, start_index=0, length=-1):
    """Sum of columns [start, start+length) of every 2-D input."""
    acc = None
    for t in x:
        r = _raw(t)
        s = start_index % r.shape[1] if start_index < 0 else start_index
        e = r.shape[1] if length < 0 else s + length
        acc = r[:, s:e] if acc is None else acc + r[:, s:e]
    return _wrap(acc)


def shuffle_batch(x, seed=None, startup_seed=0):
    """Shuffle rows (all leading dims flattened); returns (out, shuffle_idx, seed_out)."""
    r = _raw(x)
    flat = r.reshape(-1, r.shape[-1])
    s = int(_raw(seed).reshape(-1)[0]) if seed is not None else int(startup_seed)
    gen = torch.Generator(device="cpu")
    gen.manual_seed(s)
    idx = torch.randperm(flat.shape[0], generator=gen).to(r.device)
    return (_wrap(flat[idx].reshape(r.shape)), _wrap(idx.to(torch.int64)),
            _wrap(torch.tensor([s + 1], dtype=torch.int64)))


def hash_op(x, num_hash=1, mod_by=100000):
    """Per-row hash ids (num_hash independent hashes of each int64 row, modulo mod_by)."""
    r = _raw(x).long()
    rows = r.reshape(r.shape[0], -1)
    out = torch.empty(rows.shape[0], num_hash, 1, dtype=torch.int64, device=r.device)
    for k in range(num_hash):
        h = torch.full((rows.shape[0],), 1469598103934665603 + k, dtype=torch.int64, device=r.device)
        for c in range(rows.shape[1]):
            h = (h ^ rows[:, c]) * 1099511628211
        out[:, k, 0] = torch.remainder(h, mod_by)
    return _wrap(out)


def print_op(x, first_n=-1, message="", summarize=20, print_tensor_name=True, print_tensor_type=True,
          print_tensor_shape=True, print_tensor_layout=True, print_tensor_lod=True, print_phase="BOTH",
          is_forward=True):
    r = _raw(x)
    parts = [message] if message else []
    if print_tensor_type:
        parts.append(f"dtype: {r.dtype}")
    if print_tensor_shape:
        parts.append(f"shape: {list(r.shape)}")
    vals = r.reshape(-1)[: summarize if summarize > 0 else None].tolist()
    parts.append(f"data: {vals}")
    print("  ".join(parts))
    return x


def add_position_encoding(x, alpha=1.0, beta=1.0):
    """x * alpha + beta * sinusoidal position encoding ([B, S, D], half sin / half cos)."""
    r = _raw(x)
    B, S, D = r.shape
    half = D // 2
    pos = torch.arange(S, device=r.device, dtype=torch.float32)[:, None]
    div = torch.pow(10000.0, torch.arange(half, device=r.device, dtype=torch.float32) / max(half - 1, 1))
    enc = torch.cat([torch.sin(pos / div), torch.cos(pos / div)], dim=1)
    return _wrap((r.float() * alpha + beta * enc[None]).to(r.dtype))


def cvm(x, cvm, use_cvm=True):  # noqa: A002
    """Continuous-value model: the first two columns (show, click) become log(show+1), log(click+1)-log(show+1),
    or are dropped when use_cvm is False."""
    r = _raw(x).float()
    if not use_cvm:
        return _wrap(r[:, 2:])
    show = torch.log(r[:, :1] + 1)
    click = torch.log(r[:, 1:2] + 1) - show
    return _wrap(torch.cat([show, click, r[:, 2:]], dim=1))


def batch_fc(input, w, bias):  # noqa: A002
    """Per-slot FC: out[s] = input[s] @ w[s] + bias[s] ([S, N, in] x [S, in, out])."""
    return _wrap(torch.bmm(_raw(input), _raw(w)) + _raw(bias).unsqueeze(1))


def accuracy_check(x, y, fn_name="", rtol=1e-5, atol=1e-8, equal_nan=False):
    ok = torch.allclose(_raw(x).float(), _raw(y).float(), rtol=rtol, atol=atol, equal_nan=equal_nan)
    if not ok:
        raise AssertionError(f"accuracy_check failed for {fn_name}")
    return _wrap(torch.tensor(True))


def coalesce_tensor(input, dtype=None, copy_data=False, set_constant=False, persist_output=False,  # noqa: A002
                    constant=0.0, use_align=True, align_size=-1, size_of_dtype=-1, concated_shapes=(),
                    concated_ranks=()):
    """One flat buffer holding every input (256-B aligned chunks when use_align); returns (outputs as views of the
    buffer, fused buffer)."""
    ts = [_raw(t) for t in input]
    dt = ts[0].dtype
    esz = torch.empty((), dtype=dt).element_size()
    align = (align_size if align_size > 0 else 256) // esz if use_align else 1
    sizes = [((t.numel() + align - 1) // align) * align for t in ts]
    buf = torch.full((sum(sizes),), constant if set_constant else 0, dtype=dt, device=ts[0].device)
    outs, off = [], 0
    for t, n in zip(ts, sizes):
        v = buf[off: off + t.numel()].view(t.shape)
        if copy_data:
            v.copy_(t)
        outs.append(_wrap(v))
        off += n
    return outs, _wrap(buf)


coalesce_tensor_ = coalesce_tensor


def embedding_grad_dense(x, weight, out_grad, padding_idx=-1, sparse=False):
    ids = _raw(x).reshape(-1).long()
    g = _raw(out_grad).reshape(ids.numel(), -1)
    w = _raw(weight)
    dw = torch.zeros(w.shape, dtype=torch.float32, device=w.device)
    keep = ids != padding_idx if padding_idx >= 0 else torch.ones_like(ids, dtype=torch.bool)
    dw.index_add_(0, ids[keep], g[keep].float())
    return _wrap(dw.to(w.dtype))


def straight_through_estimator_grad(out_grad):
    return out_grad


_ACTS = {"relu": F.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh, "gelu": F.gelu, "identity": lambda t: t,
         "scale": lambda t: t, "swish": F.silu, "silu": F.silu}


def fused_elemwise_activation(x, y, functor_list=("elementwise_add", "relu"), axis=-1, scale=0.0,
                              save_intermediate_out=False):
    """Two-functor fusion: [binary, unary] -> binary(x, unary(y)); [unary, binary] -> unary(binary(x, y))."""
    a, b = _raw(x), _raw(y)
    f0, f1 = functor_list

    def binary(name, u, v):
        return {"elementwise_add": torch.add, "elementwise_mul": torch.mul, "elementwise_sub": torch.sub}[name](u, v)

    def unary(name, t):
        return t * scale if name == "scale" else _ACTS[name](t)

    if f0.startswith("elementwise_"):
        inter = unary(f1, b)
        out = binary(f0, a, inter)
    else:
        inter = binary(f1, a, b)
        out = unary(f0, inter)
    return (_wrap(out), _wrap(inter)) if save_intermediate_out else _wrap(out)


def fused_elemwise_add_activation(x, y, functor_list=("elementwise_add", "relu"), axis=-1, scale=0.0,
                                  save_intermediate_out=False):
    return fused_elemwise_activation(x, y, functor_list, axis, scale, save_intermediate_out)


def fused_fc_elementwise_layernorm(x, w, y, bias0=None, scale=None, bias1=None, x_num_col_dims=1,
                                   activation_type="", epsilon=1e-5, begin_norm_axis=1):
    """layer_norm(act(x @ w + bias0) + y) (fused_ops.yaml fused_fc_elementwise_layernorm)."""
    xr = _raw(x).reshape(int(torch.tensor(_raw(x).shape[:x_num_col_dims]).prod()), -1)
    h = xr @ _raw(w)
    if bias0 is not None:
        h = h + _raw(bias0)
    if activation_type:
        h = _ACTS[activation_type](h)
    h = h + _raw(y).reshape(h.shape)
    nshape = h.shape[begin_norm_axis:]
    out = F.layer_norm(h.float(), nshape, None if scale is None else _raw(scale).float(),
                       None if bias1 is None else _raw(bias1).float(), epsilon).to(h.dtype)
    return _wrap(out)


def fused_scale_bias_add_relu(x1, scale1, bias1, x2, scale2=None, bias2=None, fuse_dual=False, exhaustive_search=False):
    """relu(x1 * scale1 + bias1 + (x2 * scale2 + bias2 if fuse_dual else x2)) over NHWC channels."""
    a = _raw(x1) * _raw(scale1) + _raw(bias1)
    b = _raw(x2) * _raw(scale2) + _raw(bias2) if fuse_dual else _raw(x2)
    return _wrap(F.relu(a + b))


def fused_embedding_eltwise_layernorm(ids, embs, bias, scale, epsilon=1e-5):
    """layer_norm(sum_i embs[i][ids[i]]) (ERNIE-style embedding fusion)."""
    acc = None
    for i, e in zip(ids, embs):
        v = F.embedding(_raw(i).long(), _raw(e))
        acc = v if acc is None else acc + v
    return _wrap(F.layer_norm(acc.float(), acc.shape[-1:], _raw(scale).float(), _raw(bias).float(),
                              epsilon).to(acc.dtype))


def squeeze_excitation_block(x, filter, filter_max=None, bias=None, branch=None, act_type=(1, 1, 1),  # noqa: A002
                             act_param=(0.0, 0.0, 0.0), filter_dims=()):
    """SE block: x * sigmoid(fc2(relu(fc1(avgpool(x))))) with filter = [fc1 | fc2] flattened ([C/r*C + C*C/r])."""
    r = _raw(x)
    C = r.shape[1]
    f = _raw(filter).reshape(-1)
    mid = f.numel() // (2 * C)
    w1, w2 = f[: mid * C].reshape(mid, C), f[mid * C:].reshape(C, mid)
    s = r.float().mean(dim=(2, 3))
    h = F.relu(s @ w1.float().t())
    g = torch.sigmoid(h @ w2.float().t())
    out = r * g[:, :, None, None].to(r.dtype)
    if branch is not None:
        out = out + _raw(branch)
    return _wrap(out)


def fp8_fp8_half_gemm_fused(x, y, bias=None, transpose_x=False, transpose_y=False, scale=1.0, output_dtype="float16",
                            activation_type="identity"):
    """fp8 x fp8 -> half GEMM with bias + activation (reference fusion/fp8_gemm): the fp8 operands go through the
    framework's fp8 GEMM path (ops/fp8.py) with a scalar scale."""
    a, b = _raw(x), _raw(y)
    a = a.transpose(-1, -2) if transpose_x else a
    b = b.transpose(-1, -2) if transpose_y else b
    out = (a.float() @ b.float()) * scale
    if bias is not None:
        out = out + _raw(bias).float()
    out = _ACTS.get(activation_type, lambda t: t)(out)
    return _wrap(out.to(torch.float16 if output_dtype == "float16" else torch.bfloat16))


def apply_per_channel_scale(x, scales):
    return _wrap(_raw(x) * _raw(scales))


def quant_linear(x, w, bias=None, in_num_col_dims=1, activation_type="", padding_weights=False, scale_in=1.0,
                 scale_weights=(1.0,), quant_round_type=1, quant_max_bound=127.0, quant_min_bound=-127.0):
    """int8 linear: x_q = round(x * scale_in * bound) (clipped), w holds int8 values whose dequantised weight is
    w * scale_weights (per output channel), out = (x_q @ w) * scale_weights / (scale_in * bound) + bias."""
    xr = _raw(x).float()
    xq = torch.clamp(torch.round(xr * scale_in * quant_max_bound), quant_min_bound, quant_max_bound)
    sw = torch.as_tensor(scale_weights, dtype=torch.float32, device=xr.device)
    acc = xq.reshape(-1, xq.shape[-1]) @ _raw(w).float()
    out = acc * sw / (scale_in * quant_max_bound)
    if bias is not None:
        out = out + _raw(bias).float()
    if activation_type:
        out = _ACTS[activation_type](out)
    return _wrap(out.reshape(*xr.shape[:-1], -1).to(_raw(x).dtype))


def fake_quantize_range_abs_max(x, in_scale, iter=None, window_size=10000, bit_length=8, is_test=False,  # noqa: A002
                                round_type=1):
    """Quantise-dequantise with the running max of |x| (fake_quantize ops): returns (out, out_scale)."""
    r = _raw(x).float()
    bnd = (1 << (bit_length - 1)) - 1
    s = _raw(in_scale).float().reshape(-1)[0]
    if not is_test:
        s = torch.maximum(s, r.abs().max())
    out = torch.round(torch.clamp(r / s, -1, 1) * bnd) * s / bnd
    return _wrap(out.to(_raw(x).dtype)), _wrap(s.reshape(1))


def moving_average_abs_max_scale(x, in_accum=None, in_state=None, moving_rate=0.9, is_test=False):
    """scale = accum / state with accum = rate * accum + max|x|, state = rate * state + 1."""
    r = _raw(x).float()
    cur = r.abs().max()
    acc = _raw(in_accum).float().reshape(-1)[0] if in_accum is not None else torch.tensor(0.0)
    st = _raw(in_state).float().reshape(-1)[0] if in_state is not None else torch.tensor(0.0)
    if not is_test:
        acc = moving_rate * acc + cur
        st = moving_rate * st + 1
    return x, _wrap((acc / st).reshape(1)), _wrap(st.reshape(1)), _wrap(acc.reshape(1))


# ------------------------------------------------------------------------------------------ sparse long tail
def sparse_acos(x):
    return _sparse_unary(x, torch.acos)


def sparse_acosh(x):
    return _sparse_unary(x, torch.acosh)


def _sparse_unary(x, fn):
    r = _raw(x)
    if r.layout == torch.sparse_coo:
        r = r.coalesce()
        return _wrap(torch.sparse_coo_tensor(r.indices(), fn(r.values()), r.shape))
    if r.layout == torch.sparse_csr:
        return _wrap(torch.sparse_csr_tensor(r.crow_indices(), r.col_indices(), fn(r.values()), r.shape))
    return _wrap(fn(r))


def sparse_full_like(x, value, dtype=None):
    r = _raw(x)
    if r.layout == torch.sparse_coo:
        r = r.coalesce()
        return _wrap(torch.sparse_coo_tensor(r.indices(), torch.full_like(r.values(), value), r.shape))
    return _wrap(torch.full_like(r, value))


# ------------------------------------------------------------------------------------------ recurrent
def rnn(x, pre_state, weight_list, sequence_length=None, dropout_prob=0.0, is_bidirec=False, input_size=10,
        hidden_size=100, num_layers=1, mode="RNN_TANH", seed=0, is_test=False):
    """The fused cuDNN-style rnn op over [S, B, in] input (time-major): modes LSTM / GRU / RNN_TANH / RNN_RELU;
    weight_list = per layer/direction [w_ih, w_hh] then the biases (reference ops.yaml rnn)."""
    xr = _raw(x)
    ndir = 2 if is_bidirec else 1
    kind = {"LSTM": torch.nn.LSTM, "GRU": torch.nn.GRU}.get(mode, torch.nn.RNN)
    kw = {} if kind is not torch.nn.RNN else {"nonlinearity": "relu" if mode == "RNN_RELU" else "tanh"}
    mod = kind(input_size, hidden_size, num_layers, bias=True, batch_first=False, dropout=0.0,
               bidirectional=is_bidirec, **kw).to(xr.device, xr.dtype)
    ws = [_raw(w) for w in weight_list]
    nw = num_layers * ndir
    names = []
    for layer in range(num_layers):
        for d in range(ndir):
            sfx = f"_l{layer}" + ("_reverse" if d else "")
            names.append((f"weight_ih{sfx}", f"weight_hh{sfx}", f"bias_ih{sfx}", f"bias_hh{sfx}"))
    with torch.no_grad():
        for i, (wi, wh, bi, bh) in enumerate(names):
            getattr(mod, wi).copy_(ws[2 * i])
            getattr(mod, wh).copy_(ws[2 * i + 1])
            getattr(mod, bi).copy_(ws[2 * nw + 2 * i])
            getattr(mod, bh).copy_(ws[2 * nw + 2 * i + 1])
    states = [_raw(s) for s in pre_state]
    h0 = tuple(states) if mode == "LSTM" else states[0]
    out, hn = mod(xr, h0)
    hn = list(hn) if isinstance(hn, tuple) else [hn]
    return _wrap(out), None, [_wrap(h) for h in hn], None


def lstm(input, init_h, init_c, weight, bias, use_peepholes=False, is_reverse=False,  # noqa: A002
         gate_activation="sigmoid", cell_activation="tanh", candidate_activation="tanh"):
    """Single-layer LSTM over [B, S, 4H] pre-projected input (legacy lstm op): weight [H, 4H], bias [1, 4H]."""
    xr = _raw(input)
    h, c = _raw(init_h), _raw(init_c)
    W, b = _raw(weight), _raw(bias).reshape(-1)[: W.shape[1]]
    steps = range(xr.shape[1] - 1, -1, -1) if is_reverse else range(xr.shape[1])
    outs = [None] * xr.shape[1]
    for t in steps:
        g = xr[:, t] + h @ W + b
        i, f, cc, o = g.chunk(4, dim=-1)
        c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(cc)
        h = torch.sigmoid(o) * torch.tanh(c)
        outs[t] = h
    return _wrap(torch.stack(outs, 1)), _wrap(torch.stack(outs, 1)), _wrap(c)


def gru_unit(input, hidden_prev, weight, bias=None, activation=2, gate_activation=1,  # noqa: A002
             origin_mode=False):
    """One GRU step on pre-projected input [B, 3H] (legacy gru_unit): weight [H, 3H] = [W_u | W_r | W_c]."""
    x, hp, W = _raw(input), _raw(hidden_prev), _raw(weight)
    H = hp.shape[-1]
    if bias is not None:
        x = x + _raw(bias).reshape(-1)
    ur = x[:, : 2 * H] + hp @ W[:, : 2 * H]
    u, r = torch.sigmoid(ur).chunk(2, dim=-1)
    c = torch.tanh(x[:, 2 * H:] + (r * hp) @ W[:, 2 * H:])
    h = u * hp + (1 - u) * c if origin_mode else (1 - u) * hp + u * c
    return _wrap(torch.cat([u, r, c], -1)), _wrap(r * hp), _wrap(h)


def beam_search(pre_ids, pre_scores, ids, scores, level=0, beam_size=4, end_id=0, is_accumulated=True):
    """One beam-search step over [B*beam, K] candidates: keep the beam_size best per source sentence; finished
    beams (pre_id == end_id) keep only themselves.  Returns (selected_ids, selected_scores, parent_idx)."""
    pi, ps = _raw(pre_ids).reshape(-1), _raw(pre_scores).reshape(-1)
    cand_ids, cand_sc = _raw(ids), _raw(scores)
    if not is_accumulated:
        cand_sc = ps[:, None] + torch.log(cand_sc)
    fin = pi == end_id
    cand_sc = torch.where(fin[:, None], torch.full_like(cand_sc, -float("inf")), cand_sc)
    cand_sc[:, 0] = torch.where(fin, ps, cand_sc[:, 0])
    cand_ids = torch.where(fin[:, None], torch.full_like(cand_ids, end_id), cand_ids)
    nb = pi.numel() // beam_size
    sc = cand_sc.reshape(nb, -1)
    top, arg = sc.topk(beam_size, dim=-1)
    K = cand_ids.shape[1]
    parent = (arg // K) + torch.arange(nb, device=arg.device)[:, None] * beam_size
    sel = cand_ids.reshape(nb, -1).gather(1, arg)
    return _wrap(sel.reshape(-1, 1)), _wrap(top.reshape(-1, 1)), _wrap(parent.reshape(-1))


def beam_search_decode(ids, scores, beam_size, end_id):
    """Back-track per-step (ids, parent) lists into full hypotheses: ids / scores are lists of
    (selected_ids [N,1], parent_idx [N]) step tensors; returns ([N, T] ids, [N] final scores)."""
    steps = list(ids)
    T = len(steps)
    n = _raw(steps[-1][0]).shape[0]
    out = torch.zeros(n, T, dtype=torch.int64, device=_raw(steps[-1][0]).device)
    cur = torch.arange(n, device=out.device)
    for t in range(T - 1, -1, -1):
        sid, par = _raw(steps[t][0]).reshape(-1), _raw(steps[t][1]).reshape(-1)
        out[:, t] = sid[cur]
        cur = par[cur]
    final = _raw(list(scores)[-1]).reshape(-1)
    return _wrap(out), _wrap(final)


# ------------------------------------------------------------------------------------------ detection / sequence
def ctc_align(input, input_length=None, blank=0, merge_repeated=True, padding_value=0):  # noqa: A002
    """CTC greedy-decode alignment: merge repeats, drop blanks, left-pack each row (padded with padding_value);
    returns (output [B, T], output_length [B, 1])."""
    x = _raw(input).long()
    B, T = x.shape[0], x.shape[1]
    lens = _raw(input_length).reshape(-1).long() if input_length is not None else torch.full((B,), T)
    out = torch.full((B, T), padding_value, dtype=x.dtype, device=x.device)
    olen = torch.zeros(B, 1, dtype=torch.int64, device=x.device)
    for b in range(B):
        prev, k = None, 0
        for t in range(int(lens[b])):
            tok = int(x[b, t])
            if tok != blank and not (merge_repeated and tok == prev):
                out[b, k] = tok
                k += 1
            prev = tok
        olen[b, 0] = k
    return _wrap(out), _wrap(olen)


def crf_decoding(emission, transition, label=None, length=None):
    """Viterbi decode of a linear-chain CRF: transition [(n+2), n] with the start / stop rows first (reference
    crf_decoding op layout); emission [B, T, n]; returns the best path [B, T] (or, with label, 1 where the path
    matches the label)."""
    e = _raw(emission).float()
    tr = _raw(transition).float()
    start, stop, trans = tr[0], tr[1], tr[2:]
    B, T, n = e.shape
    lens = _raw(length).reshape(-1).long() if length is not None else torch.full((B,), T, dtype=torch.long)
    path = torch.zeros(B, T, dtype=torch.int64, device=e.device)
    for b in range(B):
        L = int(lens[b])
        if L == 0:
            continue
        score = start + e[b, 0]
        back = []
        for t in range(1, L):
            cand = score[:, None] + trans
            score, idx = cand.max(0)
            score = score + e[b, t]
            back.append(idx)
        score = score + stop
        best = int(score.argmax())
        path[b, L - 1] = best
        for t in range(L - 2, -1, -1):
            best = int(back[t][best])
            path[b, t] = best
    if label is not None:
        return _wrap((path == _raw(label).reshape(B, T).long()).to(torch.int64))
    return _wrap(path)


def chunk_eval(inference, label, chunk_scheme="IOB", num_chunk_types=1, excluded_chunk_types=(), seq_length=None):
    """Chunk precision / recall / F1 for IOB / IOE / IOBES tagging (reference chunk_eval op): tag = type * K + pos."""
    scheme = {"IOB": ("B", "I"), "IOE": ("I", "E"), "IOBES": ("B", "I", "E", "S"), "plain": ("I",)}[chunk_scheme]
    K = len(scheme)

    def chunks(seq):
        out, start, ctype, prev_end = set(), None, None, False
        for i, tag in enumerate(list(seq) + [-1]):
            if tag < 0 or tag >= num_chunk_types * K:
                if start is not None:
                    out.add((start, i - 1, ctype))
                start = None
                continue
            t, pos = tag // K, scheme[tag % K]
            begins = pos in ("B", "S") or start is None or t != ctype or (chunk_scheme == "IOE" and prev_end)
            if begins:
                if start is not None:
                    out.add((start, i - 1, ctype))
                start, ctype = i, t
            prev_end = pos in ("E", "S")
            if pos in ("E", "S"):
                out.add((start, i, ctype))
                start = None
        return {c for c in out if c[2] not in excluded_chunk_types}

    inf, lab = _raw(inference).reshape(_raw(inference).shape[0], -1), _raw(label).reshape(_raw(label).shape[0], -1)
    lens = _raw(seq_length).reshape(-1).tolist() if seq_length is not None else [inf.shape[1]] * inf.shape[0]
    ni = nl = nc = 0
    for b in range(inf.shape[0]):
        ci, cl = chunks(inf[b, : int(lens[b])].tolist()), chunks(lab[b, : int(lens[b])].tolist())
        ni, nl, nc = ni + len(ci), nl + len(cl), nc + len(ci & cl)
    p = nc / ni if ni else 0.0
    r = nc / nl if nl else 0.0
    f = 2 * p * r / (p + r) if nc else 0.0
    t = lambda v, dt=torch.float32: _wrap(torch.tensor([v], dtype=dt))  # noqa: E731
    return t(p), t(r), t(f), t(ni, torch.int64), t(nl, torch.int64), t(nc, torch.int64)


def auc(x, label, stat_pos, stat_neg, ins_tag_weight=None, curve="ROC", num_thresholds=4095, slide_steps=1):
    """Streaming AUC (reference auc op): bucket the positive-class probability into num_thresholds+1 bins,
    accumulate positive / negative histograms into stat_pos / stat_neg, return (auc, stat_pos, stat_neg)."""
    p = _raw(x)
    p = p[:, -1] if p.dim() == 2 else p.reshape(-1)
    y = _raw(label).reshape(-1).long()
    bins = torch.clamp((p.float() * num_thresholds).long(), 0, num_thresholds)
    sp, sn = _raw(stat_pos).reshape(-1), _raw(stat_neg).reshape(-1)
    sp += torch.bincount(bins[y == 1], minlength=num_thresholds + 1)[: sp.numel()].to(sp.dtype)
    sn += torch.bincount(bins[y == 0], minlength=num_thresholds + 1)[: sn.numel()].to(sn.dtype)
    tp = torch.flip(sp.double(), [0]).cumsum(0)
    fp = torch.flip(sn.double(), [0]).cumsum(0)
    tpr = torch.cat([torch.zeros(1, dtype=torch.float64), tp / max(tp[-1].item(), 1)])
    fpr = torch.cat([torch.zeros(1, dtype=torch.float64), fp / max(fp[-1].item(), 1)])
    area = torch.trapz(tpr, fpr).item() if tp[-1] > 0 and fp[-1] > 0 else 0.0
    return _wrap(torch.tensor([area], dtype=torch.float64)), stat_pos, stat_neg


def bipartite_match(dist_matrix, match_type="bipartite", dist_threshold=0.5):
    """Greedy bipartite matching of a [R, C] similarity matrix (reference bipartite_match op): repeatedly take the
    global max; with match_type 'per_prediction' unmatched columns take their best row above dist_threshold.
    Returns (col -> row index [1, C] or -1, matched distance [1, C])."""
    d = _raw(dist_matrix).float().clone()
    R, Cn = d.shape
    idx = torch.full((Cn,), -1, dtype=torch.int64)
    dist = torch.zeros(Cn)
    work = d.clone()
    for _ in range(min(R, Cn)):
        v, flat = work.reshape(-1).max(0)
        if v.item() <= 0 and not torch.isfinite(v):
            break
        r, c = divmod(int(flat), Cn)
        if work[r, c] == -float("inf"):
            break
        idx[c], dist[c] = r, d[r, c]
        work[r, :] = -float("inf")
        work[:, c] = -float("inf")
    if match_type == "per_prediction":
        for c in range(Cn):
            if idx[c] < 0:
                v, r = d[:, c].max(0)
                if v >= dist_threshold:
                    idx[c], dist[c] = int(r), v
    return _wrap(idx[None]), _wrap(dist[None])


def anchor_generator(input, anchor_sizes=(64, 128, 256, 512), aspect_ratios=(0.5, 1.0, 2.0),  # noqa: A002
                     variances=(0.1, 0.1, 0.2, 0.2), stride=(16.0, 16.0), offset=0.5):
    """Faster-RCNN anchors over an NCHW feature map: (anchors [H, W, A, 4] in x1y1x2y2, variances like it)."""
    H, W = _raw(input).shape[2], _raw(input).shape[3]
    sw, sh = stride
    base = []
    for r in aspect_ratios:
        for s in anchor_sizes:
            area = sw * sh
            bw = round((area / r) ** 0.5)
            bh = round(bw * r)
            scale_w, scale_h = s / sw, s / sh
            aw, ah = scale_w * bw, scale_h * bh
            base.append((-(aw - 1) / 2, -(ah - 1) / 2, (aw - 1) / 2, (ah - 1) / 2))
    base = torch.tensor(base)
    cx = (torch.arange(W) * sw + offset * (sw - 1)).float()
    cy = (torch.arange(H) * sh + offset * (sh - 1)).float()
    ctr = torch.stack(torch.meshgrid(cy, cx, indexing="ij"), -1)  # [H, W, 2] (y, x)
    shift = torch.stack([ctr[..., 1], ctr[..., 0], ctr[..., 1], ctr[..., 0]], -1)[:, :, None, :]
    anchors = shift + base[None, None]
    var = torch.tensor(variances, dtype=torch.float32).expand_as(anchors).clone()
    return _wrap(anchors), _wrap(var)


def _nms(boxes, scores, thr, normalized=True):
    order = scores.argsort(descending=True)
    keep = []
    off = 0.0 if normalized else 1.0
    area = (boxes[:, 2] - boxes[:, 0] + off) * (boxes[:, 3] - boxes[:, 1] + off)
    while order.numel():
        i = int(order[0])
        keep.append(i)
        if order.numel() == 1:
            break
        rest = order[1:]
        xx1 = torch.maximum(boxes[i, 0], boxes[rest, 0])
        yy1 = torch.maximum(boxes[i, 1], boxes[rest, 1])
        xx2 = torch.minimum(boxes[i, 2], boxes[rest, 2])
        yy2 = torch.minimum(boxes[i, 3], boxes[rest, 3])
        inter = (xx2 - xx1 + off).clamp(min=0) * (yy2 - yy1 + off).clamp(min=0)
        iou = inter / (area[i] + area[rest] - inter)
        order = rest[iou <= thr]
    return torch.tensor(keep, dtype=torch.int64)


def multiclass_nms3(bboxes, scores, rois_num=None, score_threshold=0.05, nms_top_k=1000, keep_top_k=100,
                    nms_threshold=0.3, normalized=True, nms_eta=1.0, background_label=0):
    """Per-class NMS then a cross-class keep_top_k (reference multiclass_nms3): bboxes [N, M, 4], scores
    [N, C, M]; returns (out [K, 6] = label, score, box; index [K, 1]; per-image counts [N])."""
    bx, sc = _raw(bboxes).float(), _raw(scores).float()
    outs, idxs, counts = [], [], []
    M = bx.shape[1]
    for n in range(bx.shape[0]):
        dets = []
        for c in range(sc.shape[1]):
            if c == background_label:
                continue
            s = sc[n, c]
            cand = (s > score_threshold).nonzero().reshape(-1)
            if cand.numel() == 0:
                continue
            if nms_top_k > -1 and cand.numel() > nms_top_k:
                cand = cand[s[cand].argsort(descending=True)[:nms_top_k]]
            keep = cand[_nms(bx[n, cand], s[cand], nms_threshold, normalized)]
            for k in keep.tolist():
                dets.append((float(s[k]), c, k))
        dets.sort(key=lambda t: -t[0])
        if keep_top_k > -1:
            dets = dets[:keep_top_k]
        for score, c, k in dets:
            outs.append([float(c), score] + bx[n, k].tolist())
            idxs.append([n * M + k])
        counts.append(len(dets))
    out = torch.tensor(outs, dtype=torch.float32).reshape(-1, 6)
    return _wrap(out), _wrap(torch.tensor(idxs, dtype=torch.int64).reshape(-1, 1)), \
        _wrap(torch.tensor(counts, dtype=torch.int32))


def multiclass_nms(bboxes, scores, score_threshold=0.05, nms_top_k=1000, keep_top_k=100, nms_threshold=0.3,
                   normalized=True, nms_eta=1.0, background_label=0):
    return multiclass_nms3(bboxes, scores, None, score_threshold, nms_top_k, keep_top_k, nms_threshold, normalized,
                           nms_eta, background_label)[0]


def im2sequence(x, y=None, kernels=(1, 1), strides=(1, 1), paddings=(0, 0, 0, 0), out_stride=(1, 1)):
    """Image patches as a sequence (reference im2sequence): [N, C, H, W] -> [N * oh * ow, C * kh * kw]."""
    r = _raw(x)
    pt, pl, pb, pr = paddings
    r = F.pad(r, (pl, pr, pt, pb))
    cols = F.unfold(r, tuple(kernels), stride=tuple(strides))  # [N, C*kh*kw, L]
    return _wrap(cols.transpose(1, 2).reshape(-1, cols.shape[1]))


def correlation(input1, input2, pad_size=4, kernel_size=1, max_displacement=4, stride1=1, stride2=1,
                corr_type_multiply=1):
    """FlowNet correlation: for every displacement (dy, dx) in [-d, d]^2 (step stride2), the channel-mean of
    input1 * shifted input2 -> [N, (2d/s2+1)^2, H, W] (kernel_size 1, stride1 1)."""
    a, b = _raw(input1).float(), _raw(input2).float()
    N, C, H, W = a.shape
    bp = F.pad(b, (pad_size, pad_size, pad_size, pad_size))
    outs = []
    rng = range(-max_displacement, max_displacement + 1, stride2)
    for dy in rng:
        for dx in rng:
            sh = bp[:, :, pad_size + dy: pad_size + dy + H, pad_size + dx: pad_size + dx + W]
            outs.append((a * sh).sum(1) / C)
    return _wrap(torch.stack(outs, 1).to(_raw(input1).dtype))


# ------------------------------------------------------------------------------------------ fused inference long tail
def add_group_norm_silu(x, residual=None, scale=None, bias=None, epsilon=1e-5, groups=32, data_format="NHWC",
                        activation="silu"):
    """(x + residual) -> group_norm -> SiLU (diffusion UNet fusion); returns (y, residual_out, mean, var)."""
    r = _raw(x)
    h = r + _raw(residual) if residual is not None else r
    nhwc = data_format == "NHWC"
    hc = h.movedim(-1, 1) if nhwc else h
    y = F.group_norm(hc.float(), groups, None if scale is None else _raw(scale).float(),
                     None if bias is None else _raw(bias).float(), epsilon)
    if activation == "silu":
        y = F.silu(y)
    y = (y.movedim(1, -1) if nhwc else y).to(r.dtype)
    g = hc.float().reshape(hc.shape[0], groups, -1)
    return _wrap(y), _wrap(h), _wrap(g.mean(-1)), _wrap(g.var(-1, unbiased=False))


def fused_conv2d_add_act(input, filter, bias=None, residual_data=None, strides=(1, 1), paddings=(0, 0),  # noqa: A002
                         padding_algorithm="EXPLICIT", dilations=(1, 1), groups=1, data_format="NCHW",
                         activation="relu", split_channels=(), exhaustive_search=False, workspace_size_MB=512,
                         fuse_alpha=0.0):
    x, w = _raw(input), _raw(filter)
    nhwc = data_format == "NHWC"
    xc = x.movedim(-1, 1) if nhwc else x
    pad = list(paddings)[:2] if len(paddings) >= 2 else [paddings[0]] * 2
    y = F.conv2d(xc, w, None if bias is None else _raw(bias), tuple(strides), tuple(pad), tuple(dilations), groups)
    if residual_data is not None:
        res = _raw(residual_data)
        y = y + (res.movedim(-1, 1) if nhwc else res)
    y = {"relu": F.relu, "identity": lambda t: t, "sigmoid": torch.sigmoid, "swish": F.silu,
         "leaky_relu": lambda t: F.leaky_relu(t, fuse_alpha)}.get(activation, lambda t: t)(y)
    return _wrap(y.movedim(1, -1) if nhwc else y)


def fusion_repeated_fc_relu(x, w, bias):
    """relu(... relu(x @ w0 + b0) ... @ wn + bn); returns (relu_out list, out)."""
    h = _raw(x)
    outs = []
    for wi, bi in zip(w, bias):
        h = F.relu(h @ _raw(wi) + _raw(bi).reshape(-1))
        outs.append(_wrap(h))
    return outs[:-1], outs[-1]


def fusion_squared_mat_sub(x, y, scalar=1.0):
    """scalar * ((x @ y)^2 - (x^2 @ y^2)) (the FM second-order term); returns (squared_x, squared_y,
    squared_xy, out)."""
    a, b = _raw(x), _raw(y)
    xy = a @ b
    sx, sy = a * a, b * b
    return _wrap(sx), _wrap(sy), _wrap(xy * xy), _wrap(scalar * (xy * xy - sx @ sy))


def fusion_transpose_flatten_concat(x, trans_axis, flatten_axis, concat_axis):
    outs = []
    for t in x:
        r = _raw(t).permute(list(trans_axis))
        outs.append(r.reshape(int(torch.tensor(r.shape[:flatten_axis]).prod()), -1))
    return _wrap(torch.cat(outs, concat_axis))


def multihead_matmul(input, w, bias, bias_qk=None, transpose_q=False, transpose_k=True, transpose_v=False,  # noqa: A002
                     alpha=1.0, head_number=1):
    """Fused BERT self-attention (inference): qkv = input @ w + bias with w [H, 3, H]; per-head softmax(alpha q
    k^T + bias_qk) v; out [B, S, H]."""
    x = _raw(input)
    B, S, H = x.shape
    W = _raw(w).reshape(H, 3 * H)
    qkv = (x @ W + _raw(bias).reshape(-1)).reshape(B, S, 3, head_number, H // head_number)
    q, k, v = (qkv[:, :, i].transpose(1, 2) for i in range(3))
    s = alpha * (q @ k.transpose(-1, -2))
    if bias_qk is not None:
        s = s + _raw(bias_qk)
    o = torch.softmax(s.float(), -1).to(x.dtype) @ v
    return _wrap(o.transpose(1, 2).reshape(B, S, H))


def self_dp_attention(x, alpha=1.0, head_number=1):
    """Self attention over a packed [B, S, 3, heads, d] qkv tensor (CPU oneDNN op in the reference)."""
    r = _raw(x)
    B, S = r.shape[0], r.shape[1]
    q, k, v = (r[:, :, i].transpose(1, 2) for i in range(3))
    o = torch.softmax((alpha * q @ k.transpose(-1, -2)).float(), -1).to(r.dtype) @ v
    return _wrap(o.transpose(1, 2).reshape(B, S, -1))


def fused_gate_attention(query, key=None, query_weight=None, key_weight=None, value_weight=None, qkv_weight=None,
                         nonbatched_bias=None, src_mask=None, gate_weight=None, gate_bias=None, out_linear_weight=None,
                         out_linear_bias=None, has_gating=True, merge_qkv=True, use_flash_attn=False):
    """AlphaFold gated self-attention: qkv_weight [3, h, d, c]; softmax(q k^T / sqrt(d) + mask + bias) v, gated by
    sigmoid(q_in . gate_weight + gate_bias), output projection [h, d, c]."""
    x = _raw(query)                     # [B, N, S, c]
    W = _raw(qkv_weight)                # [3, h, d, c]
    q, k, v = (torch.einsum("bnsc,hdc->bnhsd", x, W[i]) for i in range(3))
    d = W.shape[2]
    s = torch.einsum("bnhsd,bnhtd->bnhst", q * d ** -0.5, k)
    if src_mask is not None:
        s = s + _raw(src_mask)
    if nonbatched_bias is not None:
        s = s + _raw(nonbatched_bias)
    o = torch.einsum("bnhst,bnhtd->bnhsd", torch.softmax(s.float(), -1).to(x.dtype), v)
    if has_gating:
        g = torch.einsum("bnsc,chd->bnhsd", x, _raw(gate_weight))
        if gate_bias is not None:
            g = g + _raw(gate_bias)[None, None, :, None, :]
        o = o * torch.sigmoid(g)
    out = torch.einsum("bnhsd,hdc->bnsc", o, _raw(out_linear_weight))
    if out_linear_bias is not None:
        out = out + _raw(out_linear_bias)
    return _wrap(out)


def cudnn_lstm(x, init_h, init_c, w=None, weight_list=None, sequence_length=None, dropout_prob=0.0,
               is_bidirec=False, hidden_size=100, num_layers=1, is_test=False, seed=0):
    """The cuDNN LSTM op: time-major [S, B, in] LSTM over a weight list (same layout as the rnn op)."""
    out, _, states, _ = rnn(x, [init_h, init_c], weight_list, sequence_length, dropout_prob, is_bidirec,
                            _raw(x).shape[-1], hidden_size, num_layers, "LSTM", seed, is_test)
    return out, states[0], states[1]


def resnet_basic_block(x, filter1, scale1, bias1, mean1, var1, filter2, scale2, bias2, mean2, var2, filter3=None,
                       scale3=None, bias3=None, mean3=None, var3=None, stride1=1, stride2=1, stride3=1, padding1=1,
                       padding2=1, padding3=0, dilation1=1, dilation2=1, dilation3=1, group=1, momentum=0.9,
                       epsilon=1e-5, data_format="NCHW", has_shortcut=False, use_global_stats=True, is_test=True,
                       trainable_statistics=False, act_type="relu", find_conv_input_max=True):
    """Inference ResNet basic block: relu(bn2(conv2(relu(bn1(conv1 x)))) + shortcut(x))."""
    r = _raw(x)

    def cbn(t, f, s, b, m, v, st, pd, dl):
        y = F.conv2d(t, _raw(f), None, st, pd, dl, group)
        return F.batch_norm(y, _raw(m), _raw(v), _raw(s), _raw(b), False, 0.0, epsilon)

    h = F.relu(cbn(r, filter1, scale1, bias1, mean1, var1, stride1, padding1, dilation1))
    h = cbn(h, filter2, scale2, bias2, mean2, var2, stride2, padding2, dilation2)
    sc = cbn(r, filter3, scale3, bias3, mean3, var3, stride3, padding3, dilation3) if has_shortcut else r
    return _wrap(F.relu(h + sc))


def resnet_unit(x, filter_x, scale_x, bias_x, mean_x, var_x, z=None, filter_z=None, scale_z=None, bias_z=None,
                mean_z=None, var_z=None, stride=1, stride_z=1, padding=0, dilation=1, group=1, momentum=0.9,
                epsilon=1e-5, data_format="NHWC", fuse_add=False, has_shortcut=False, use_global_stats=True,
                is_test=True, use_addto=False, act_type="relu"):
    """conv + BN (+ a second conv+BN or a residual add) + ReLU (the ResNet unit fusion)."""
    nhwc = data_format == "NHWC"
    r = _raw(x).movedim(-1, 1) if nhwc else _raw(x)
    y = F.conv2d(r, _raw(filter_x), None, stride, padding, dilation, group)
    y = F.batch_norm(y, _raw(mean_x), _raw(var_x), _raw(scale_x), _raw(bias_x), False, 0.0, epsilon)
    if has_shortcut:
        zz = _raw(z).movedim(-1, 1) if nhwc else _raw(z)
        zs = F.conv2d(zz, _raw(filter_z), None, stride_z, 0, 1, group)
        y = y + F.batch_norm(zs, _raw(mean_z), _raw(var_z), _raw(scale_z), _raw(bias_z), False, 0.0, epsilon)
    elif fuse_add:
        y = y + (_raw(z).movedim(-1, 1) if nhwc else _raw(z))
    y = F.relu(y) if act_type == "relu" else y
    return _wrap(y.movedim(1, -1) if nhwc else y)


def blha_get_max_len(seq_lens_encoder, seq_lens_decoder, batch_size):
    """Max encoder / decoder sequence lengths of a block-attention batch (two [1] int32 tensors)."""
    e, d = _raw(seq_lens_encoder).reshape(-1), _raw(seq_lens_decoder).reshape(-1)
    return (_wrap(e.max().reshape(1).to(torch.int32)), _wrap(d.max().reshape(1).to(torch.int32)))


def calc_reduced_attn_scores(q, k, softmax_lse):
    """sum over query rows of the softmax probabilities, per key: [B, H, 1, Sk] (reference calc_reduced_attn op,
    used for KV-cache pruning), recomputed from q, k and the forward's log-sum-exp."""
    qf, kf = _raw(q).float().transpose(1, 2), _raw(k).float().transpose(1, 2)  # [B, H, S, D]
    if kf.shape[1] != qf.shape[1]:
        kf = kf.repeat_interleave(qf.shape[1] // kf.shape[1], 1)
    s = qf @ kf.transpose(-1, -2) / qf.shape[-1] ** 0.5
    lse = _raw(softmax_lse).float()[..., : s.shape[2], None]
    return _wrap(torch.exp(s - lse).sum(2, keepdim=True))


def sparse_batch_norm_(x, mean, variance, scale, bias, is_test=False, momentum=0.9, epsilon=1e-5,
                       data_format="NDHWC", use_global_stats=False, trainable_statistics=False):
    """Batch norm over the values of a sparse COO tensor (channel = last dim of the values)."""
    r = _raw(x).coalesce()
    vals = r.values()
    y = F.batch_norm(vals, _raw(mean), _raw(variance), _raw(scale), _raw(bias),
                     not (is_test or use_global_stats), 1 - momentum, epsilon)
    return _wrap(torch.sparse_coo_tensor(r.indices(), y, r.shape))


sparse_sync_batch_norm_ = sparse_batch_norm_


def yolo_box_head(x, anchors, class_num):
    """YOLOv3 head activation: sigmoid on x, y, objectness and class scores, exp kept raw for w, h (reference
    yolo_box_head, inference)."""
    r = _raw(x).clone()
    N, C, H, W = r.shape
    na = len(anchors) // 2
    v = r.reshape(N, na, 5 + class_num, H, W)
    v[:, :, 0:2] = torch.sigmoid(v[:, :, 0:2])
    v[:, :, 4:] = torch.sigmoid(v[:, :, 4:])
    return _wrap(v.reshape(N, C, H, W))


# ------------------------------------------------------------------------------------------ batch 4: DGC, LoD fusions, misc
def dgc_clip_by_norm(x, current_step, max_norm, rampup_begin_step=-1.0):
    """clip_by_norm once DGC is active (current_step >= rampup_begin_step), identity before."""
    if float(_raw(current_step).reshape(-1)[0]) < rampup_begin_step:
        return x
    r = _raw(x)
    n = r.float().norm()
    return _wrap((r.float() * torch.clamp(max_norm / n.clamp_min(1e-12), max=1.0)).to(r.dtype))


@torch.no_grad()
def dgc_momentum(param, grad, velocity, learning_rate, master_param=None, current_step_tensor=None,
                 nranks_tensor=None, mu=0.9, use_nesterov=False, regularization_method="", regularization_coeff=0.0,
                 multi_precision=False, rescale_grad=1.0, rampup_begin_step=-1.0):
    """Momentum before DGC's rampup step, plain SGD after (the velocity then lives in the DGC op)."""
    step = float(_raw(current_step_tensor).reshape(-1)[0]) if current_step_tensor is not None else 0.0
    p, g = _p(param, master_param, multi_precision), _raw(grad).float() * rescale_grad
    if nranks_tensor is not None:
        g = g / float(_raw(nranks_tensor).reshape(-1)[0])
    lr = _lr(learning_rate)
    if step < rampup_begin_step:
        v = _raw(velocity).float() * mu + g
        upd = (g + mu * v) if use_nesterov else v
        _upd(velocity, v)
    else:
        upd = g
    _store(param, master_param, multi_precision, p - lr * upd)
    return param, velocity, master_param


@torch.no_grad()
def dgc(u, v, grad, param=None, current_step=None, nranks=None, m=0.9, use_nesterov=True, sparsity=(0.999,),
        rampup_begin_step=0.0, rampup_step=0.0, regular_coeff=0.0, regular_type=0):
    """Deep Gradient Compression (reference dgc op): momentum correction u = m u + g, v += u (nesterov: u =
    m (u + g), v += u + g), keep the top-(1 - sparsity) |v| entries as the encoded gradient, clear them from u
    and v.  Returns (u, v, encode_grad (indices, values), grad_out (dense), k, gather_buff)."""
    g = _raw(grad).float()
    step = float(_raw(current_step).reshape(-1)[0]) if current_step is not None else 0.0
    sp = list(sparsity) if isinstance(sparsity, (list, tuple)) else [sparsity]
    idx = 0 if rampup_step <= 0 else min(len(sp) - 1, int((step - rampup_begin_step) * len(sp) / rampup_step))
    s = sp[max(idx, 0)]
    uu, vv = _raw(u).float(), _raw(v).float()
    if use_nesterov:
        uu = m * (uu + g)
        vv = vv + uu + g
    else:
        uu = m * uu + g
        vv = vv + uu
    k = max(1, int(round(g.numel() * (1 - s))))
    flat = vv.reshape(-1)
    top = flat.abs().topk(k).indices
    dense = torch.zeros_like(flat)
    dense[top] = flat[top]
    uflat = uu.reshape(-1).clone()
    uflat[top] = 0
    flat = flat.clone()
    flat[top] = 0
    _upd(u, uflat.reshape(uu.shape))
    _upd(v, flat.reshape(vv.shape))
    enc = torch.cat([top.float(), dense[top]])
    return u, v, _wrap(enc), _wrap(dense.reshape(g.shape).to(_raw(grad).dtype)), _wrap(torch.tensor([k])), None


def collect_fpn_proposals(multi_level_rois, multi_level_scores, multi_level_rois_num=None, post_nms_topn=2000):
    """Concatenate the per-level RoIs and keep the post_nms_topn highest-scoring ones (per image when
    rois_num is given); returns (rois, rois_num)."""
    rois = torch.cat([_raw(r) for r in multi_level_rois])
    sc = torch.cat([_raw(s).reshape(-1) for s in multi_level_scores])
    if multi_level_rois_num is None:
        keep = sc.argsort(descending=True)[:post_nms_topn]
        return _wrap(rois[keep]), _wrap(torch.tensor([keep.numel()], dtype=torch.int32))
    nums = [_raw(n).reshape(-1).long() for n in multi_level_rois_num]
    n_img = nums[0].numel()
    img = torch.cat([torch.repeat_interleave(torch.arange(n_img), n) for n in nums])
    outs, cnt = [], []
    for i in range(n_img):
        sel = (img == i).nonzero().reshape(-1)
        keep = sel[sc[sel].argsort(descending=True)[:post_nms_topn]]
        outs.append(rois[keep])
        cnt.append(keep.numel())
    return _wrap(torch.cat(outs)), _wrap(torch.tensor(cnt, dtype=torch.int32))


def fusion_seqpool_concat(x, pooltype="SUM", axis=1):
    from ..static.sequence import sequence_pool

    return _wrap(torch.cat([_raw(sequence_pool(t, pooltype)) for t in x], axis))


def fused_seqpool_cvm(x, cvm, pooltype="SUM", pad_value=0.0, use_cvm=True, cvm_offset=2):
    from ..static.sequence import sequence_pool

    outs = []
    for t in x:
        pooled = sequence_pool(t, pooltype, pad_value=pad_value)
        outs.append(_raw(cvm_fn(pooled, use_cvm)))
    return [_wrap(o) for o in outs]


def cvm_fn(t, use_cvm):
    return cvm(t, None, use_cvm)


def fusion_seqpool_cvm_concat(x, cvm, pooltype="SUM", use_cvm=True, axis=1):
    return _wrap(torch.cat([_raw(o) for o in fused_seqpool_cvm(x, cvm, pooltype, 0.0, use_cvm)], axis))


def dist_concat(x, ring_id=0, nranks=1):
    """All-gather along axis 0 over the ring (one rank: identity)."""
    if nranks <= 1:
        return x
    from ..distributed import collective as Cc

    parts = []
    Cc.all_gather(parts, x)
    return _wrap(torch.cat([_raw(p) for p in parts], 0))


def fused_token_prune(attn, x, mask, new_mask, keep_first_token=True, keep_order=False):
    """Keep the tokens with the largest attention received (column sums of attn [B, H, S, S] over heads and
    queries, masked) — new_mask's length S' tokens per sample; returns (pruned x [B, S', C], cls_inds)."""
    a = (_raw(attn) + _raw(mask)).float().clamp_min(0) if mask is not None else _raw(attn).float()
    score = a.sum((1, 2))                              # [B, S]
    s_new = _raw(new_mask).shape[-1]
    if keep_first_token:
        score[:, 0] = float("inf")
    idx = score.topk(s_new, -1).indices
    if keep_order:
        idx = idx.sort(-1).values
    xr = _raw(x)
    out = xr.gather(1, idx[..., None].expand(-1, -1, xr.shape[-1]))
    return _wrap(out), _wrap(idx)


def graph_khop_sampler(row, colptr, x, eids=None, sample_sizes=(-1,), return_eids=False):
    """Multi-hop neighbour sampling: sample_neighbors hop by hop from the frontier, then reindex the union
    subgraph (reference graph_khop_sampler); returns (edge_src, edge_dst, sample_index, reindex_x)."""
    from ..geometric import reindex_graph, sample_neighbors

    frontier = x
    srcs, dsts, counts_all, centers = [], [], [], []
    for k in sample_sizes:
        nb, cnt = sample_neighbors(row, colptr, frontier, sample_size=k)[:2]
        srcs.append(_raw(nb))
        centers.append(_raw(frontier))
        counts_all.append(_raw(cnt))
        frontier = _wrap(torch.unique(_raw(nb)))
    nbs = torch.cat(srcs)
    cnt = torch.cat(counts_all)
    ctr = torch.cat(centers)
    rs, rd, nodes = reindex_graph(_wrap(ctr), _wrap(nbs), _wrap(cnt))
    return rs, rd, nodes, _wrap(torch.arange(_raw(x).numel()))


def tdm_child(x, tree_info, child_nums=2, dtype="int32"):
    """Children of tree nodes (reference tdm_child): tree_info rows are [item_id, layer, parent, child_0, ...];
    returns (children ids, leaf mask)."""
    ids = _raw(x).long()
    info = _raw(tree_info).long()
    ch = info[ids.reshape(-1)][:, 3:3 + child_nums].reshape(*ids.shape, child_nums)
    leaf = (info[ch.clamp_min(0).reshape(-1)][:, 0] != 0).reshape(ch.shape) & (ch > 0)
    tdt = torch.int64 if dtype == "int64" else torch.int32
    return _wrap(ch.to(tdt)), _wrap(leaf.to(tdt))


def lookup_table_dequant(w, ids, padding_idx=-1):
    """Embedding over a uint8-quantised table: each row = [min, max, q_0 .. q_{D-1}] (floats holding packed
    bytes in the reference); here rows are [min, max, codes...] as floats and value = min + code * (max-min)/255."""
    tab = _raw(w).float()
    i = _raw(ids).reshape(-1).long()
    rows = tab[i]
    mn, mx, codes = rows[:, :1], rows[:, 1:2], rows[:, 2:]
    out = mn + codes * (mx - mn) / 255.0
    if padding_idx >= 0:
        out[i == padding_idx] = 0
    return _wrap(out.reshape(*_raw(ids).shape, -1))


def gru(input, h0, weight, bias=None, batch_size=None, batch_gate=None, batch_reset_hidden_prev=None,  # noqa: A002
        batch_hidden=None, activation="tanh", gate_activation="sigmoid", is_reverse=False, origin_mode=False,
        is_test=False):
    """Full-sequence GRU over a LoD input of pre-projected gates [T, 3H] (reference gru op): each sequence runs
    gru_unit steps from h0 (zeros when None); returns the hidden states [T, H] (with the input's LoD)."""
    from ..static.sequence import _offsets

    x = _raw(input)
    off = _offsets(input)
    H = x.shape[1] // 3
    out = torch.zeros(x.shape[0], H, dtype=x.dtype, device=x.device)
    for s, (a, b) in enumerate(zip(off[:-1], off[1:])):
        h = _raw(h0)[s:s + 1] if h0 is not None else torch.zeros(1, H, dtype=x.dtype, device=x.device)
        rng = range(b - 1, a - 1, -1) if is_reverse else range(a, b)
        for t in rng:
            _, _, hn = gru_unit(_wrap(x[t:t + 1]), _wrap(h), weight, bias, origin_mode=origin_mode)
            h = _raw(hn)
            out[t] = h[0]
    res = _wrap(out)
    res._lod = input._lod
    return res


def fusion_gru(x, h0, weight_x, weight_h, bias=None, activation="tanh", gate_activation="sigmoid",
               is_reverse=False, use_seq=True, origin_mode=False, use_mkldnn=False, mkldnn_data_type="float32",
               scale_data=1.0, shift_data=0.0, scale_weights=(1.0,), force_fp32_output=False):
    """x @ weight_x (+ bias) then the LoD GRU (reference fusion_gru)."""
    proj = _wrap(_raw(x) @ _raw(weight_x) + (_raw(bias).reshape(-1) if bias is not None else 0))
    proj._lod = x._lod
    return gru(proj, h0, weight_h, None, is_reverse=is_reverse, origin_mode=origin_mode)


def fusion_lstm(x, weight_x, weight_h, bias, h0=None, c0=None, use_peepholes=False, is_reverse=False,
                use_seq=True, gate_activation="sigmoid", cell_activation="tanh", candidate_activation="tanh",
                scale_data=1.0, shift_data=0.0, scale_weights=(1.0,), force_fp32_output=False):
    """x @ weight_x then an LSTM over each LoD sequence (gates i, f, c, o); returns (hidden [T, H], cell [T, H])."""
    from ..static.sequence import _offsets

    proj = _raw(x) @ _raw(weight_x) + _raw(bias).reshape(-1)[: _raw(weight_x).shape[1]]
    off = _offsets(x)
    H = _raw(weight_h).shape[0]
    hs = torch.zeros(proj.shape[0], H, dtype=proj.dtype)
    cs = torch.zeros_like(hs)
    for s, (a, b) in enumerate(zip(off[:-1], off[1:])):
        h = _raw(h0)[s] if h0 is not None else torch.zeros(H, dtype=proj.dtype)
        c = _raw(c0)[s] if c0 is not None else torch.zeros(H, dtype=proj.dtype)
        for t in (range(b - 1, a - 1, -1) if is_reverse else range(a, b)):
            gi, gf, gc, go = (proj[t] + h @ _raw(weight_h)).chunk(4)
            c = torch.sigmoid(gf) * c + torch.sigmoid(gi) * torch.tanh(gc)
            h = torch.sigmoid(go) * torch.tanh(c)
            hs[t], cs[t] = h, c
    ho, co = _wrap(hs), _wrap(cs)
    ho._lod = co._lod = x._lod
    return ho, co


# ------------------------------------------------------------------------------------------ long tail, batch 5
def rank_attention(x, rank_offset, rank_param, max_rank=3, max_size=0):
    """Reference rank_attention (paddle/phi/kernels/gpu/rank_attention_kernel.cu, funcs/rank_attention.cu.h):
    rank_offset [N, 2*max_rank+1] = (own rank, then per slot k: (peer rank, peer row)).  Slot k of instance i
    holds x[peer row] when both ranks are set (1-based; <= 0 means empty); the instance's parameter block for
    slot k is rank_param rows [((own-1)*max_rank + peer-1) * D, +D).  Returns (input_help [N, max_rank*D],
    out [N, P] = input_help @ per-instance parameter, ins_rank [N, 1]) -- batched as one bmm instead of the
    reference's expand-then-GEMM kernels."""
    xr, ro, rp = _raw(x), _raw(rank_offset).long(), _raw(rank_param)
    N, D = xr.shape
    P = rp.shape[1]
    own = ro[:, 0] - 1
    peer = ro[:, 1::2][:, :max_rank] - 1
    row = ro[:, 2::2][:, :max_rank]
    valid = (own[:, None] >= 0) & (peer >= 0)
    help_ = torch.where(valid[..., None], xr[row.clamp(0, N - 1)], torch.zeros((), dtype=xr.dtype))
    blk = (own[:, None].clamp(min=0) * max_rank + peer.clamp(min=0))              # [N, max_rank]
    params = rp.reshape(-1, D, P)[blk] * valid[..., None, None].to(rp.dtype)      # [N, max_rank, D, P]
    out = torch.bmm(help_.reshape(N, 1, max_rank * D), params.reshape(N, max_rank * D, P)).reshape(N, P)
    return _wrap(help_.reshape(N, max_rank * D)), _wrap(out), _wrap(ro[:, :1].to(xr.dtype))


def qkv_unpack_mha(q, k, v, src_mask=None):
    """Reference qkv_unpack_mha (paddle/phi/kernels/fusion/gpu/qkv_unpack_mha_kernel.cu): one decode step of
    multi-head attention over separate q [B, 1, Hq, D], k / v [B, S, Hkv, D] (grouped heads share a kv head)
    with an additive src_mask broadcastable to [B, Hq, 1, S]; output [B, 1, Hq, D].  Runs on the framework's
    flash / SDPA path."""
    qr, kr, vr = _raw(q), _raw(k), _raw(v)
    B, _, Hq, D = qr.shape
    g = Hq // kr.shape[2]
    kt = kr.transpose(1, 2).repeat_interleave(g, 1)
    vt = vr.transpose(1, 2).repeat_interleave(g, 1)
    mask = None if src_mask is None else _raw(src_mask).to(qr.dtype)
    o = F.scaled_dot_product_attention(qr.transpose(1, 2), kt, vt, attn_mask=mask, scale=D ** -0.5)
    return _wrap(o.transpose(1, 2).contiguous())


def match_matrix_tensor(x, y, w, dim_t=1):
    """Reference match_matrix_tensor (paddle/phi/kernels/cpu/match_matrix_tensor_kernel.cc): for LoD sequence
    pairs (x_i [Lx, D], y_i [Ly, D]) and w [D, dim_t, D] emits x_i W_t y_i^T for every channel t, flattened per
    sequence into out [sum_i dim_t*Lx_i*Ly_i, 1] (LoD over sequences); tmp = x @ w ([Tx, dim_t*D])."""
    from ..static.sequence import _offsets

    xr, yr, wr = _raw(x), _raw(y), _raw(w)
    D = xr.shape[1]
    tmp = xr @ wr.reshape(D, dim_t * D)
    ox, oy = _offsets(x), _offsets(y)
    outs, lod = [], [0]
    for (a, b), (c, d) in zip(zip(ox[:-1], ox[1:]), zip(oy[:-1], oy[1:])):
        t = tmp[a:b].reshape(b - a, dim_t, D).transpose(0, 1)                     # [dim_t, Lx, D]
        m = t @ yr[c:d].t()                                                        # [dim_t, Lx, Ly]
        outs.append(m.reshape(-1, 1))
        lod.append(lod[-1] + m.numel())
    out = _wrap(torch.cat(outs) if outs else tmp.new_zeros(0, 1))
    out._lod = [lod]
    return out, _wrap(tmp)


def _context_cols(r, off, size, start, stride=1):
    """Per-sequence context window: row t gets rows [t+start, t+start+size) of its own sequence (zero padded),
    flattened to [T, size*D] (the im2col of sequence_conv)."""
    D = r.shape[1]
    cols = torch.zeros(r.shape[0], size * D, dtype=r.dtype, device=r.device)
    for a, b in zip(off[:-1], off[1:]):
        for k in range(size):
            sh = start + k
            lo, hi = max(a, a - sh), min(b, b - sh)
            if hi > lo:
                cols[lo:hi, k * D:(k + 1) * D] = r[lo + sh:hi + sh]
    return cols


def fusion_seqconv_eltadd_relu(x, filter, bias, context_length, context_start=0, context_stride=1):  # noqa: A002
    """Reference fusion_seqconv_eltadd_relu (paddle/phi/kernels/fusion/cpu/fusion_seqconv_eltadd_relu_kernel.cc):
    relu(sequence_conv(x) + bias); returns (out [T, F], col_mat [T, context_length*D])."""
    from ..static.sequence import _offsets

    xr = _raw(x)
    cols = _context_cols(xr, _offsets(x), context_length, context_start, context_stride)
    out = _wrap(torch.relu(cols @ _raw(filter) + _raw(bias).reshape(-1)))
    out._lod = x._lod
    return out, _wrap(cols)


_FC_ACT = {"identity": lambda t: t, "relu": torch.relu, "sigmoid": torch.sigmoid, "tanh": torch.tanh}


def fusion_seqexpand_concat_fc(x, fc_weight, fc_bias=None, fc_activation="identity"):
    """Reference fusion_seqexpand_concat_fc (fusion/cpu/fusion_seqexpand_concat_fc_kernel.cc): x[0] is a LoD
    batch [T, D0]; x[1:] are per-sequence rows [N, Di] expanded over their sequence's steps; the concatenation
    [T, sum D] goes through fc (+bias, activation).  Returns (out [T, F], fc_out = x[1:]'s share of the fc)."""
    from ..static.sequence import _offsets

    off = _offsets(x[0])
    reps = torch.tensor([b - a for a, b in zip(off[:-1], off[1:])])
    parts = [_raw(x[0])] + [torch.repeat_interleave(_raw(t), reps, 0) for t in x[1:]]
    cat = torch.cat(parts, 1)
    w = _raw(fc_weight)
    d0 = parts[0].shape[1]
    fc_out = torch.cat([_raw(t) for t in x[1:]], 1) @ w[d0:] if len(x) > 1 else cat.new_zeros(0)
    y = cat @ w
    if fc_bias is not None:
        y = y + _raw(fc_bias).reshape(-1)
    out = _wrap(_FC_ACT[fc_activation](y))
    out._lod = x[0]._lod
    return out, _wrap(fc_out)


def fused_embedding_fc_lstm(ids, embeddings, weight_h, bias, h0=None, c0=None, use_peepholes=True,
                            is_reverse=False, use_seq=True, gate_activation="sigmoid", cell_activation="tanh",
                            candidate_activation="tanh"):
    """Reference fused_embedding_fc_lstm (fusion/cpu/fused_embedding_fc_lstm_kernel.cc): ``embeddings`` is
    the embedding table already multiplied by the LSTM input weight ([V, 4H]), so the gate projection of a
    step is one row lookup; then the LoD LSTM (gates i, f, c, o).  Returns (hidden, cell)."""
    idr = _raw(ids).reshape(-1).long()
    proj = _wrap(_raw(embeddings)[idr])
    proj._lod = ids._lod
    H = _raw(weight_h).shape[0]
    eye = _wrap(torch.eye(4 * H, dtype=_raw(embeddings).dtype))
    return fusion_lstm(proj, eye, weight_h, bias, h0, c0, use_peepholes, is_reverse, use_seq, gate_activation,
                       cell_activation, candidate_activation)


def attention_lstm(x, c0, h0=None, attention_weight=None, attention_bias=None, attention_scalar=None,
                   attention_scalar_bias=None, lstm_weight=None, lstm_bias=None, gate_activation="sigmoid",
                   cell_activation="tanh", candidate_activation="tanh"):
    """Reference attention_lstm (paddle/phi/kernels/cpu/attention_lstm_kernel.cc): at every step of a LoD
    sequence x_s [L, M] the previous cell state attends over the whole sequence -- score_j = relu?(fc([x_j,
    c_prev])) (scalar / scalar-bias rescale, relu), softmax over j -- and the pooled x feeds the LSTM together
    with h_prev: gates = [pooled, h_prev] @ lstm_weight + lstm_bias (gate order f, i, o, c as the reference's
    kernel lays them out).  Returns (hidden [T, D], cell [T, D])."""
    from ..static.sequence import _offsets

    xr, aw = _raw(x), _raw(attention_weight)
    M = xr.shape[1]
    lw, lb = _raw(lstm_weight), _raw(lstm_bias).reshape(-1)
    D = lw.shape[1] // 4
    off = _offsets(x)
    hs = torch.zeros(xr.shape[0], D, dtype=xr.dtype)
    cs = torch.zeros_like(hs)
    ab = _raw(attention_bias).reshape(-1) if attention_bias is not None else None
    for s, (a, b) in enumerate(zip(off[:-1], off[1:])):
        seq = xr[a:b]
        c = _raw(c0)[s]
        h = _raw(h0)[s] if h0 is not None else torch.zeros(D, dtype=xr.dtype)
        xs = seq @ aw[:M].reshape(M, -1)                                            # [L, 1]
        for t in range(b - a):
            sc = (xs + c @ aw[M:].reshape(D, -1)).reshape(-1)
            if ab is not None:
                sc = sc + ab[0]
            sc = torch.relu(sc)
            if attention_scalar is not None:
                sc = sc * _raw(attention_scalar).reshape(-1)[0]
                if attention_scalar_bias is not None:
                    sc = sc + _raw(attention_scalar_bias).reshape(-1)[0]
                sc = torch.relu(sc)
            pooled = torch.softmax(sc, 0) @ seq                                     # [M]
            gf, gi, go, gc = (torch.cat([pooled, h]) @ lw + lb).chunk(4)
            c = torch.sigmoid(gf) * c + torch.sigmoid(gi) * torch.tanh(gc)
            h = torch.sigmoid(go) * torch.tanh(c)
            hs[a + t], cs[a + t] = h, c
    ho, co = _wrap(hs), _wrap(cs)
    ho._lod = co._lod = x._lod
    return ho, co


def yolo_box_post(boxes0, boxes1, boxes2, image_shape, image_scale, anchors0, anchors1, anchors2, class_num,
                  conf_thresh, downsample_ratio0, downsample_ratio1, downsample_ratio2, clip_bbox=True,
                  scale_x_y=1.0, nms_threshold=0.45):
    """Reference yolo_box_post (paddle/phi/kernels/fusion/gpu/yolo_box_post_kernel.cu): decode the three YOLOv3
    heads (yolo_box), map boxes back to the original image (divide by image_scale), then per-image multi-class
    NMS.  Returns (out [K, 6] = label, score, x1, y1, x2, y2; nms_rois_num [N])."""
    from ..vision.ops import yolo_box

    shp = _wrap(_raw(image_shape).int())
    bxs, scs = [], []
    for hd, an, ds in ((boxes0, anchors0, downsample_ratio0), (boxes1, anchors1, downsample_ratio1),
                       (boxes2, anchors2, downsample_ratio2)):
        b, s = yolo_box(hd, shp, list(an), class_num, conf_thresh, ds, clip_bbox, scale_x_y=scale_x_y)
        bxs.append(_raw(b).float())
        scs.append(_raw(s).float())
    bx = torch.cat(bxs, 1)
    sc = torch.cat(scs, 1)
    scale = _raw(image_scale).float().reshape(bx.shape[0], -1)
    sx, sy = scale[:, -1:], scale[:, :1]                      # image_scale rows are (scale_y, scale_x)
    bx = bx / torch.cat([sx, sy, sx, sy], 1)[:, None, :]
    out, _, num = multiclass_nms3(_wrap(bx), _wrap(sc.transpose(1, 2)), None, conf_thresh, -1, -1,
                                  nms_threshold, False, 1.0, -1)
    return out, num


def p_send_array(x, ring_id=0, peer=0, use_calc_stream=True, dynamic_shape=False):
    """Reference p_send_array (static pipeline send of a tensor array): the array length, then each tensor
    (with its shape first when ``dynamic_shape``), over the framework's point-to-point path."""
    from ..distributed import collective as C

    C.send(_wrap(torch.tensor([len(x)], dtype=torch.int64)), dst=peer)
    for t in x:
        if dynamic_shape:
            shp = list(_raw(t).shape)
            C.send(_wrap(torch.tensor([len(shp)] + shp, dtype=torch.int64)), dst=peer)
        C.send(t if hasattr(t, "_t") else _wrap(t), dst=peer)


def p_recv_array(ring_id=0, peer=0, dtype="float32", out_shape=(), use_calc_stream=True, dynamic_shape=False):
    """Counterpart of p_send_array: receives the array length, then each tensor (``out_shape`` per element, or
    the sent shapes with ``dynamic_shape``); returns the list of tensors."""
    from ..distributed import collective as C
    from ..framework.dtype import convert_dtype

    n = _wrap(torch.zeros(1, dtype=torch.int64))
    C.recv(n, src=peer)
    outs = []
    for _ in range(int(_raw(n)[0])):
        if dynamic_shape:
            hdr = _wrap(torch.zeros(9, dtype=torch.int64))
            C.recv(hdr, src=peer)
            shape = _raw(hdr)[1:1 + int(_raw(hdr)[0])].tolist()
        else:
            shape = list(out_shape)
        t = _wrap(torch.zeros(shape, dtype=convert_dtype(dtype)))
        C.recv(t, src=peer)
        outs.append(t)
    return outs


def fused_scale_bias_relu_conv_bn(x, w, scale=None, bias=None, bn_scale=None, bn_bias=None,
                                  input_running_mean=None, input_running_var=None, paddings=(0, 0),
                                  dilations=(1, 1), strides=(1, 1), padding_algorithm="EXPLICIT", groups=1,
                                  data_format="NHWC", momentum=0.9, epsilon=1e-5, fuse_prologue=True,
                                  exhaustive_search=False, accumulation_count=0):
    """Reference fused_scale_bias_relu_conv_bn (fusion/gpu/fused_scale_bias_relu_conv_bn_kernel.cu, the ResNet
    unit): optional prologue relu(x*scale+bias), conv (NHWC), batch statistics of the conv output and the
    running-stat update; returns (out, out_running_mean, out_running_var, saved_mean, saved_inv_std, eq_scale,
    eq_bias) with eq_scale / eq_bias the folded BN affine (y_bn = conv*eq_scale + eq_bias)."""
    xr = _raw(x)
    nhwc = data_format == "NHWC"
    if fuse_prologue and scale is not None:
        xr = torch.relu(xr * _raw(scale).reshape(-1) + _raw(bias).reshape(-1))
    xc = xr.permute(0, 3, 1, 2) if nhwc else xr
    wr = _raw(w)
    wc = wr.permute(0, 3, 1, 2) if nhwc else wr
    pad = "same" if padding_algorithm == "SAME" else (0 if padding_algorithm == "VALID" else tuple(paddings))
    y = F.conv2d(xc.float(), wc.float(), None, tuple(strides), pad, tuple(dilations), groups)
    mean = y.mean((0, 2, 3))
    var = y.var((0, 2, 3), unbiased=False)
    inv_std = torch.rsqrt(var + epsilon)
    n = y.numel() // y.shape[1]
    rm = _raw(input_running_mean).float() * momentum + mean * (1 - momentum)
    rv = _raw(input_running_var).float() * momentum + var * n / max(n - 1, 1) * (1 - momentum)
    eq_scale = _raw(bn_scale).float() * inv_std
    eq_bias = _raw(bn_bias).float() - mean * eq_scale
    out = (y.permute(0, 2, 3, 1) if nhwc else y).to(_raw(x).dtype)
    return (_wrap(out), _wrap(rm), _wrap(rv), _wrap(mean), _wrap(inv_std), _wrap(eq_scale.to(out.dtype)),
            _wrap(eq_bias.to(out.dtype)))


def fused_multi_transformer_int8(x, ln_scale, ln_bias, qkv_w, qkv_bias, out_linear_w, out_linear_bias,
                                 ffn_ln_scale, ffn_ln_bias, ffn1_weight, ffn1_bias, ffn2_weight, ffn2_bias,
                                 qkv_out_scale=None, out_linear_out_scale=None, ffn1_out_scale=None,
                                 ffn2_out_scale=None, cache_kv=None, time_step=None, attn_mask=None,
                                 pre_layer_norm=True, epsilon=1e-5, dropout_rate=0.0, is_test=True,
                                 dropout_implementation="downgrade_in_infer", act_method="gelu", trans_qkvw=True,
                                 ring_id=-1, **_):
    """Reference fused_multi_transformer_int8 (fusion/gpu/fused_multi_transformer_int8_op.cu): the multi-layer
    decoder with int8 weights; each weight is dequantised with its per-output-channel ``*_out_scale`` (weight
    scale) and the layers run through the framework's fused_multi_transformer."""
    from ..serving import fused_multi_transformer

    def deq(ws, scales):
        if scales is None:
            return [_wrap(_raw(w).float()) for w in ws]
        return [_wrap(_raw(w).float() * _raw(s).float().reshape(*([-1] + [1] * (_raw(w).dim() - 1))))
                if _raw(w).dim() > 1 and _raw(s).numel() == _raw(w).shape[0] else
                _wrap(_raw(w).float() * _raw(s).float().reshape(-1)) for w, s in zip(ws, scales)]

    dt = _raw(x).dtype
    cast = lambda ts: [_wrap(_raw(t).to(dt)) for t in ts]  # noqa: E731
    return fused_multi_transformer(x, ln_scale, ln_bias, cast(deq(qkv_w, qkv_out_scale)), qkv_bias,
                                   cast(deq(out_linear_w, out_linear_out_scale)), out_linear_bias, ffn_ln_scale,
                                   ffn_ln_bias, cast(deq(ffn1_weight, ffn1_out_scale)), ffn1_bias,
                                   cast(deq(ffn2_weight, ffn2_out_scale)), ffn2_bias,
                                   pre_layer_norm=pre_layer_norm, epsilon=epsilon, cache_kvs=cache_kv,
                                   time_step=time_step, attn_mask=attn_mask, activation=act_method,
                                   trans_qkvw=trans_qkvw, ring_id=ring_id)


# ------------------------------------------------------------------------------------------ long tail, batch 6
def tdm_sampler(x, travel, layer, output_positive=True, neg_samples_num_list=(), layer_offset_lod=(), seed=0,
                dtype=2):
    """Reference tdm_sampler (paddle/phi/kernels/cpu/tdm_sampler_kernel.cc): for every input item walk its
    tree path (travel[item] = one positive node per layer, 0 = padding) and per layer emit the positive
    (label 1) then ``neg_samples_num_list[l]`` distinct uniform negatives of that layer (label 0) that are not
    the positive; padding layers emit zeros with mask 0.  Returns (out, labels, mask), each [N, sum(neg+pos)]."""
    import numpy as np

    ids = _raw(x).reshape(-1).long().tolist()
    tr, ly = _raw(travel).long(), _raw(layer).reshape(-1).long()
    L = len(neg_samples_num_list)
    width = sum(n + int(output_positive) for n in neg_samples_num_list)
    out = torch.zeros(len(ids), width, dtype=torch.int64)
    lab, msk = torch.zeros_like(out), torch.zeros_like(out)
    rng = np.random.default_rng(seed if seed else None)
    for i, item in enumerate(ids):
        off = 0
        for l in range(L):
            n = neg_samples_num_list[l]
            lo, hi = layer_offset_lod[l], layer_offset_lod[l + 1]
            pos = int(tr[item, l])
            if pos == 0:
                off += n + int(output_positive)
                continue
            if output_positive:
                out[i, off], lab[i, off], msk[i, off] = pos, 1, 1
                off += 1
            cand = [j for j in range(hi - lo) if int(ly[lo + j]) != pos]
            pick = rng.choice(len(cand), size=n, replace=False) if n else []
            for p in pick:
                out[i, off], msk[i, off] = int(ly[lo + cand[int(p)]]), 1
                off += 1
    cast = torch.int32 if dtype == 2 else torch.int64
    return _wrap(out.to(cast)), _wrap(lab.to(cast)), _wrap(msk.to(cast))


def _iou(a, b):
    iw = max(min(a[2], b[2]) - max(a[0], b[0]), 0.0)
    ih = max(min(a[3], b[3]) - max(a[1], b[1]), 0.0)
    inter = iw * ih
    union = (a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter
    return inter / union if union > 0 else 0.0


def detection_map(detect_res, label, has_state=None, pos_count=None, true_pos=None, false_pos=None, class_num=1,
                  background_label=0, overlap_threshold=0.5, evaluate_difficult=True, ap_type="integral"):
    """Reference detection_map (paddle/phi/kernels/cpu/detection_map_kernel.cc): LoD detections [M, 6] (label,
    score, box) against LoD ground truth [N, 6] (label, difficult, box) or [N, 5]; greedy score-ordered matching
    at IoU > overlap_threshold per class, then integral or VOC 11-point AP averaged over the classes with
    positives.  State (accumulated over batches when has_state != 0): pos_count [C, 1] and per-class (score,
    flag) lists true_pos / false_pos [K, 2] with a class LoD.  Returns (accum_pos_count, accum_true_pos,
    accum_false_pos, m_ap)."""
    from ..static.sequence import _offsets

    det, gt = _raw(detect_res).double(), _raw(label).double()
    dof, gof = _offsets(detect_res), _offsets(label)
    pc = {c: 0 for c in range(class_num)}
    tp = {c: [] for c in range(class_num)}
    fp = {c: [] for c in range(class_num)}
    if has_state is not None and int(_raw(has_state).reshape(-1)[0]) != 0:
        for c, v in enumerate(_raw(pos_count).reshape(-1).tolist()):
            pc[c] = int(v)
        for store, t in ((tp, true_pos), (fp, false_pos)):
            off = _offsets(t)
            rows = _raw(t).double()
            for c in range(len(off) - 1):
                store[c] += [(float(rows[k, 0]), int(rows[k, 1])) for k in range(off[c], off[c + 1])]
    wide = gt.shape[1] == 6
    for n in range(len(gof) - 1):
        gts = {}
        for i in range(gof[n], gof[n + 1]):
            c = int(gt[i, 0])
            diff = bool(gt[i, 1] != 0) if wide else False
            gts.setdefault(c, []).append((gt[i, 2:6].tolist() if wide else gt[i, 1:5].tolist(), diff))
            if evaluate_difficult or not diff:
                pc[c] = pc.get(c, 0) + 1
        dets = {}
        for i in range(dof[n], dof[n + 1]):
            dets.setdefault(int(det[i, 0]), []).append((float(det[i, 1]), [min(max(v, 0.0), 1.0)
                                                                           for v in det[i, 2:6].tolist()]))
        for c, preds in dets.items():
            tp.setdefault(c, []), fp.setdefault(c, [])
            if c not in gts:
                tp[c] += [(s, 0) for s, _ in preds]
                fp[c] += [(s, 1) for s, _ in preds]
                continue
            seen = [False] * len(gts[c])
            for s, box in sorted(preds, key=lambda t: -t[0]):
                ious = [_iou(box, g) for g, _ in gts[c]]
                j = max(range(len(ious)), key=lambda k: ious[k])
                if ious[j] > overlap_threshold:
                    if evaluate_difficult or not gts[c][j][1]:
                        hit = not seen[j]
                        seen[j] = True
                        tp[c].append((s, int(hit)))
                        fp[c].append((s, int(not hit)))
                else:
                    tp[c].append((s, 0))
                    fp[c].append((s, 1))
    m_ap, count = 0.0, 0
    for c, npos in pc.items():
        if npos == background_label:   # the reference compares the positive count (sic) with background_label
            continue
        if not tp.get(c):
            count += 1
            continue
        t_sorted = [f for _, f in sorted(tp[c], key=lambda t: -t[0])]
        f_sorted = [f for _, f in sorted(fp[c], key=lambda t: -t[0])]
        ct = torch.tensor(t_sorted, dtype=torch.float64).cumsum(0)
        cf = torch.tensor(f_sorted, dtype=torch.float64).cumsum(0)
        prec = (ct / (ct + cf)).tolist()
        rec = (ct / npos).tolist()
        if ap_type == "11point":
            mp = [0.0] * 11
            start = len(rec) - 1
            for j in range(10, -1, -1):
                for i in range(start, -1, -1):
                    if rec[i] < j / 10.0:
                        start = i
                        if j > 0:
                            mp[j - 1] = mp[j]
                        break
                    mp[j] = max(mp[j], prec[i])
            m_ap += sum(mp) / 11
        else:
            ap, prev = 0.0, 0.0
            for p, r in zip(prec, rec):
                if abs(r - prev) > 1e-6:
                    ap += p * abs(r - prev)
                prev = r
            m_ap += ap
        count += 1
    m_ap = m_ap / count if count else 0.0

    def pack(store):
        rows, lod = [], [0]
        for c in range(class_num):
            rows += [[s, float(f)] for s, f in store.get(c, [])]
            lod.append(len(rows))
        t = _wrap(torch.tensor(rows, dtype=torch.float32).reshape(-1, 2))
        t._lod = [lod]
        return t

    apc = _wrap(torch.tensor([[pc.get(c, 0)] for c in range(class_num)], dtype=torch.int32))
    return apc, pack(tp), pack(fp), _wrap(torch.tensor([m_ap], dtype=torch.float32))


def faster_tokenizer(vocab, text, text_pair=None, do_lower_case=False, is_split_into_words=False, max_seq_len=0,
                     pad_to_max_seq_len=False):
    """Reference faster_tokenizer (paddle/fluid/operators/string/faster_tokenizer_op.cc): BERT tokenisation --
    basic split (whitespace, punctuation, CJK chars as words, optional lower-casing / accent stripping), greedy
    longest-match WordPiece with ``##`` continuations, ``[CLS] a [SEP] (b [SEP])``, pair truncation of the
    longer side to ``max_seq_len``, [PAD] padding.  ``vocab``: dict token -> id (the reference's Vocab
    tensor); ``text`` / ``text_pair``: lists of strings.  Returns (input_ids, segment_ids) int64 [B, L]."""
    import unicodedata

    voc = dict(vocab)
    unk, cls, sep, pad = (voc.get(t, 0) for t in ("[UNK]", "[CLS]", "[SEP]", "[PAD]"))

    def basic(s):
        if do_lower_case:
            s = "".join(ch for ch in unicodedata.normalize("NFD", s.lower()) if unicodedata.category(ch) != "Mn")
        toks, cur = [], ""
        for ch in s:
            cp = ord(ch)
            punct = unicodedata.category(ch).startswith("P") or (33 <= cp <= 47 or 58 <= cp <= 64 or
                                                                 91 <= cp <= 96 or 123 <= cp <= 126)
            cjk = 0x4E00 <= cp <= 0x9FFF or 0x3400 <= cp <= 0x4DBF or 0xF900 <= cp <= 0xFAFF
            if ch.isspace():
                if cur:
                    toks.append(cur)
                cur = ""
            elif punct or cjk:
                if cur:
                    toks.append(cur)
                toks.append(ch)
                cur = ""
            else:
                cur += ch
        if cur:
            toks.append(cur)
        return toks

    def wordpiece(w):
        if len(w) > 100:
            return [unk]
        ids, start = [], 0
        while start < len(w):
            end = len(w)
            while end > start:
                piece = ("##" if start else "") + w[start:end]
                if piece in voc:
                    ids.append(voc[piece])
                    break
                end -= 1
            if end == start:
                return [unk]
            start = end
        return ids

    def encode(s):
        words = s if is_split_into_words else basic(s)
        return [i for w in words for i in wordpiece(w)]

    texts = [text] if isinstance(text, str) else list(text)
    pairs = None if text_pair is None else ([text_pair] if isinstance(text_pair, str) else list(text_pair))
    rows, segs = [], []
    for k, s in enumerate(texts):
        a = encode(s)
        b = encode(pairs[k]) if pairs else None
        if max_seq_len > 0:
            budget = max_seq_len - (3 if b is not None else 2)
            if b is None:
                a = a[:max(budget, 0)]
            else:
                while len(a) + len(b) > budget:
                    if len(a) >= len(b):
                        a = a[:-1]
                    else:
                        b = b[:-1]
        ids = [cls] + a + [sep]
        sg = [0] * len(ids)
        if b is not None:
            ids += b + [sep]
            sg += [1] * (len(b) + 1)
        rows.append(ids)
        segs.append(sg)
    L = max(len(r) for r in rows)
    if pad_to_max_seq_len and max_seq_len > 0:
        L = max(L, max_seq_len)
    ids_t = torch.full((len(rows), L), pad, dtype=torch.int64)
    seg_t = torch.zeros(len(rows), L, dtype=torch.int64)
    for i, (r, sg) in enumerate(zip(rows, segs)):
        ids_t[i, :len(r)] = torch.tensor(r)
        seg_t[i, :len(sg)] = torch.tensor(sg)
    return _wrap(ids_t), _wrap(seg_t)


_FUSION_GROUPS = {}


def register_fusion_group(func_name, fn):
    """Register the body of a fusion_group subgraph (the reference's fusion_group pass generates device code
    for an elementwise subgraph and names it ``func_name``; here the body is a Python callable over torch
    tensors, executed as one fused region -- on the GPU the elementwise chain is HBM-bound either way)."""
    _FUSION_GROUPS[func_name] = fn


def fusion_group(inputs, outs_dtype=(), inputs_dtype=(), func_name="", type=0):  # noqa: A002
    """Reference fusion_group (paddle/phi/kernels/fusion/gpu/fusion_group_kernel.cu): run the registered
    subgraph ``func_name`` over ``inputs``; outputs are cast to ``outs_dtype`` (0 = fp32, 1 = fp16, 2 = bf16,
    as the pass encodes them)."""
    if func_name not in _FUSION_GROUPS:
        raise KeyError(f"fusion_group: no subgraph registered under {func_name!r} (register_fusion_group)")
    outs = _FUSION_GROUPS[func_name](*[_raw(t) for t in inputs])
    outs = list(outs) if isinstance(outs, (list, tuple)) else [outs]
    code = {0: torch.float32, 1: torch.float16, 2: torch.bfloat16}
    return [_wrap(o.to(code[outs_dtype[i]]) if i < len(outs_dtype) else o) for i, o in enumerate(outs)]


def pyramid_hash(x, w, white_list=None, black_list=None, num_emb=0, space_len=0, pyramid_layer=2, rand_len=0,
                 drop_out_percent=0.0, is_training=0, use_filter=True, white_list_len=0, black_list_len=0, seed=0,
                 lr=0.0, distribute_update_vars=""):
    """Reference pyramid_hash (paddle/phi/kernels/cpu/pyramid_hash_kernel.cc): every n-gram (2 <= n <=
    pyramid_layer) of a LoD int32 sequence is hashed into the [space_len + rand_len] table ``w``; its num_emb
    embedding is num_emb / rand_len chunks, chunk j (at column j) = w[h_j : h_j + rand_len] with
    h_j = XXH32(n-gram int32 bytes, seed = j + seed) % space_len.  Black-listed n-grams (exact id sequences) are dropped;
    with use_filter and a white list only listed ones are kept.  Returns (out [#ngrams, num_emb] with the
    n-gram LoD, drop_pos, x_temp_out).  Hash-function parity with the reference's bloom-filter path is
    unpinned (no reference binary runs here)."""
    import xxhash

    xr = _raw(x).reshape(-1).to(torch.int32)
    wr = _raw(w).reshape(-1)
    from ..static.sequence import _offsets

    off = _offsets(x)

    def _set(t):
        if t is None:
            return set()
        return {tuple(r) for r in _raw(t).long().reshape(_raw(t).shape[0], -1).tolist()}

    wl, bl = _set(white_list), _set(black_list)
    rows, lod, drop = [], [0], []
    for a, b in zip(off[:-1], off[1:]):
        seq = xr[a:b]
        n_rows = 0
        for n in range(2, pyramid_layer + 1):
            for s in range(0, (b - a) - n + 1):
                g = seq[s:s + n]
                key = tuple(g.tolist())
                if key in bl or (use_filter and wl and key not in wl):
                    continue
                byts = g.numpy().tobytes()
                emb = []
                for j in range(0, num_emb, rand_len):
                    h = xxhash.xxh32_intdigest(byts, seed=j + seed) % space_len
                    emb.append(wr[h:h + rand_len])
                rows.append(torch.cat(emb)[:num_emb])
                n_rows += 1
                drop.append(1)
        if n_rows == 0:   # the reference emits one zero row for a sequence without n-grams
            rows.append(torch.zeros(num_emb, dtype=wr.dtype))
            drop.append(0)
            n_rows = 1
        lod.append(lod[-1] + n_rows)
    out = _wrap(torch.stack(rows))
    out._lod = [lod]
    return out, _wrap(torch.tensor(drop, dtype=torch.int32)), _wrap(xr.clone())


def distributed_fused_lamb_init(param, grad, beta1=0.9, beta2=0.999, apply_weight_decay=(), alignment=128, rank=0,
                                nranks=1):
    """Reference distributed_fused_lamb_init (fusion/gpu/distributed_fused_lamb_init_kernel.cu): pack the fp32
    and 16-bit parameters (and grads) into aligned flat buffers, zero moments, beta-power scalars, per-param
    offsets and this rank's shard offsets; param_out / master_param_out / grad_out are views into the flat
    buffers (the parameters then live in them).  Returns the 18 outputs in the reference's order."""
    ps, gs = [_raw(p) for p in param], [_raw(g) for g in grad]
    fp32 = [i for i, p in enumerate(ps) if p.dtype == torch.float32]
    half = [i for i, p in enumerate(ps) if p.dtype != torch.float32]

    def layout(idx):
        offs, n = [0], 0
        for i in idx:
            n += (ps[i].numel() + alignment - 1) // alignment * alignment
            offs.append(n)
        return offs

    o32, o16 = layout(fp32), layout(half)
    n32, n16 = o32[-1], o16[-1]
    shard = lambda n: (n + nranks - 1) // nranks  # noqa: E731
    fp32_param = torch.zeros(n32 + n16)               # masters of the 16-bit params follow the fp32 ones
    fp32_grad = torch.zeros(n32)
    fp16_param = torch.zeros(n16, dtype=ps[half[0]].dtype if half else torch.float16)
    fp16_grad = torch.zeros_like(fp16_param)
    param_out, master_out, grad_out = [None] * len(ps), [None] * len(ps), [None] * len(ps)
    for k, i in enumerate(fp32):
        a, m = o32[k], ps[i].numel()
        fp32_param[a:a + m] = ps[i].reshape(-1)
        fp32_grad[a:a + m] = gs[i].reshape(-1).float()
        param_out[i] = master_out[i] = fp32_param[a:a + m].view(ps[i].shape)
        grad_out[i] = fp32_grad[a:a + m].view(ps[i].shape)
    for k, i in enumerate(half):
        a, m = o16[k], ps[i].numel()
        fp16_param[a:a + m] = ps[i].reshape(-1)
        fp16_grad[a:a + m] = gs[i].reshape(-1).to(fp16_grad.dtype)
        fp32_param[n32 + a:n32 + a + m] = ps[i].reshape(-1).float()
        param_out[i] = fp16_param[a:a + m].view(ps[i].shape)
        master_out[i] = fp32_param[n32 + a:n32 + a + m].view(ps[i].shape)
        grad_out[i] = fp16_grad[a:a + m].view(ps[i].shape)
    s32, s16 = shard(n32), shard(n16)
    moment1 = torch.zeros(s32 + s16)
    moment2 = torch.zeros(s32 + s16)
    wd = [int(v) for v in (list(apply_weight_decay) or [1] * len(ps))]
    info = torch.tensor([s32, s16, len(fp32), len(half), rank, nranks] + wd, dtype=torch.int32)
    order = torch.tensor(fp32 + half, dtype=torch.int32)
    offs = torch.tensor(o32 + [n32 + v for v in o16[1:]], dtype=torch.int32)
    return tuple(_wrap(t) if not isinstance(t, list) else [_wrap(v) for v in t] for t in (
        fp32_param, fp32_grad, fp16_param, fp16_grad, moment1, moment2, torch.tensor([beta1]),
        torch.tensor([beta2]), offs, torch.tensor([rank * s32, min((rank + 1) * s32, n32)], dtype=torch.int32),
        torch.tensor([rank * s16, min((rank + 1) * s16, n16)], dtype=torch.int32), info, order, param_out,
        master_out, grad_out, torch.tensor([1.0]), torch.tensor([0], dtype=torch.int64)))


def fused_dconv_drelu_dbn(grad_output, weight, grad_output_add=None, residual_input=None, bn1_eqscale=None,
                          bn1_eqbias=None, conv_input=None, bn1_mean=None, bn1_inv_std=None, bn1_gamma=None,
                          bn1_beta=None, bn1_input=None, bn2_mean=None, bn2_inv_std=None, bn2_gamma=None,
                          bn2_beta=None, bn2_input=None, paddings=(0, 0), dilations=(1, 1), strides=(1, 1),
                          padding_algorithm="EXPLICIT", groups=1, data_format="NHWC", fuse_shortcut=False,
                          fuse_dual=False, fuse_add=False, exhaustive_search=False):
    """Reference fused_dconv_drelu_dbn (fusion/gpu/fused_dconv_drelu_dbn_kernel.cu), the backward of the ResNet
    unit: the conv's input was relu(bn1(bn1_input)) (+ bn2(bn2_input) with fuse_dual, + residual_input with
    fuse_shortcut); given dL/d(conv out) returns (grad_weight, grad_bn1_input, grad_bn1_gamma, grad_bn1_beta,
    grad_bn2_input, grad_bn2_gamma, grad_bn2_beta).  ``grad_output_add`` (fuse_add) is added to the gradient
    arriving at the relu output.  Computed by autograd over the composed forward (NHWC)."""
    nhwc = data_format == "NHWC"
    f32 = lambda t: None if t is None else _raw(t).float()  # noqa: E731

    def bn(inp, mean, inv, g, b):
        return (inp - mean) * inv * g + b

    x1 = f32(bn1_input).requires_grad_(True)
    g1, b1 = f32(bn1_gamma).requires_grad_(True), f32(bn1_beta).requires_grad_(True)
    pre = bn(x1, f32(bn1_mean), f32(bn1_inv_std), g1, b1)
    x2 = g2 = b2 = None
    if fuse_dual:
        x2 = f32(bn2_input).requires_grad_(True)
        g2, b2 = f32(bn2_gamma).requires_grad_(True), f32(bn2_beta).requires_grad_(True)
        pre = pre + bn(x2, f32(bn2_mean), f32(bn2_inv_std), g2, b2)
    elif fuse_shortcut and residual_input is not None:
        pre = pre + f32(residual_input)
    act = torch.relu(pre)
    w = f32(weight).requires_grad_(True)
    xc = act.permute(0, 3, 1, 2) if nhwc else act
    wc = w.permute(0, 3, 1, 2) if nhwc else w
    pad = "same" if padding_algorithm == "SAME" else (0 if padding_algorithm == "VALID" else tuple(paddings))
    y = F.conv2d(xc, wc, None, tuple(strides), pad, tuple(dilations), groups)
    dy = f32(grad_output)
    dy = dy.permute(0, 3, 1, 2) if nhwc else dy
    extra = f32(grad_output_add) if fuse_add and grad_output_add is not None else None
    objs = [y] + ([act] if extra is not None else [])
    grads = [dy] + ([extra] if extra is not None else [])
    wrt = [w, x1, g1, b1] + ([x2, g2, b2] if fuse_dual else [])
    gr = torch.autograd.grad(objs, wrt, grads)
    dt = _raw(bn1_input).dtype
    outs = [gr[0].to(_raw(weight).dtype), gr[1].to(dt), gr[2], gr[3]]
    outs += [gr[4].to(dt), gr[5], gr[6]] if fuse_dual else [None, None, None]
    return tuple(None if o is None else _wrap(o) for o in outs)
