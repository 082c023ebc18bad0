"""SPMD sharding-propagation rules (reference: paddle/phi/infermeta/spmd_rules/*.cc, exposed as
``core.get_phi_spmd_rule(name).infer_forward / infer_backward``; tests in test/auto_parallel/spmd_rules/).

A tensor's distribution is a ``dims_mapping`` (tensor axis -> process-mesh dim, -1 = replicated) plus the set of
mesh dims over which it holds PARTIAL sums.  Most rules are einsum-notation merges:

  1. every input axis gets a letter ("mk,kn->mn" for matmul, right-aligned broadcast letters for elementwise,
     size-1 broadcast axes are "1" and never sharded);
  2. per letter the inputs' mesh dims are merged: -1 yields to a sharding, two different shardings conflict and
     the letter becomes replicated;
  3. a mesh dim may shard only one letter: the first letter (in order of appearance across the inputs) keeps it;
  4. inputs are re-sharded to the merged letters, outputs take their letters' mesh dims, and a letter that is
     sharded but absent from an output (a contraction / reduction) makes that output PARTIAL on the mesh dim.

Op-specific constraints (softmax / layer-norm axes, split / concat axes, reshape axis merges, embedding vocab
sharding, ...) are applied on top, exactly where the reference's rules apply them.
"""
from __future__ import annotations

import copy
import string


# ============================================================================================ attributes
class TensorDistAttr:
    def __init__(self, dims_mapping=None, process_mesh=None, partial_dims=None):
        self.dims_mapping = list(dims_mapping) if dims_mapping is not None else []
        self.process_mesh = process_mesh
        self._partial = set(partial_dims or ())

    def _is_partial(self):
        return bool(self._partial)

    def _partial_dims(self):
        return set(self._partial)

    def _set_partial_dims(self, dims):
        self._partial = set(dims)

    def _clean_partial_dims(self, dims):
        self._partial -= set(dims)

    def __repr__(self):
        return f"TensorDistAttr(dims_mapping={self.dims_mapping}, partial={sorted(self._partial)})"


class DistTensorSpec:
    def __init__(self, shape, dist_attr=None):
        self.shape = list(shape)
        self.dist_attr = copy.deepcopy(dist_attr) if dist_attr is not None else TensorDistAttr([-1] * len(shape))

    @property
    def dims_mapping(self):
        return self.dist_attr.dims_mapping

    def set_dims_mapping(self, dm):
        self.dist_attr.dims_mapping = list(dm)

    def set_process_mesh(self, mesh):
        self.dist_attr.process_mesh = mesh


def _attr(dm, mesh, partial=()):
    return TensorDistAttr(dm, mesh, partial)


def _mesh(specs):
    for s in specs:
        if s.dist_attr.process_mesh is not None:
            return s.dist_attr.process_mesh
    return None


# ============================================================================================ merge engine
def merge_axes(notations, mappings):
    """Letters -> mesh dim after steps 2-3 of the module doc.  Tensors are scanned in order; every time a
    letter is (re)assigned a mesh dim it is appended to that dim's claimant list, and the FIRST claimant keeps
    the dim (the reference's ShardingMergeForTensors order).  Two different shardings of one letter replicate
    it (the reference raises Unimplemented there)."""
    amap = {}
    claim = {}
    for nota, dm in zip(notations, mappings):
        for ax, m in zip(nota, dm):
            if ax == "1":
                continue
            cur = amap.get(ax, -1)
            if ax not in amap or cur == -1:
                new = m
            elif m == -1 or m == cur:
                new = cur
            else:
                new = -1
            amap[ax] = new
            if new != -1:
                lst = claim.setdefault(new, [])
                if ax not in lst:
                    lst.append(ax)
    for m, axes in claim.items():
        for ax in axes[1:]:
            if amap.get(ax) == m:
                amap[ax] = -1
    return amap


def _map(nota, amap):
    return [-1 if ax == "1" else amap.get(ax, -1) for ax in nota]


def _partial(amap, out_nota):
    return {m for ax, m in amap.items() if m != -1 and ax not in out_nota}


def _letters(n, skip=""):
    return [c for c in string.ascii_lowercase if c not in skip][:n]


def _bcast_notations(shapes):
    """Right-aligned letters; an input axis of size 1 that broadcasts against a larger size is "1"."""
    nd = max(len(s) for s in shapes)
    base = _letters(nd)
    full = [max((s[i - (nd - len(s))] for s in shapes if i - (nd - len(s)) >= 0), default=1) for i in range(nd)]
    notas = []
    for s in shapes:
        off = nd - len(s)
        notas.append("".join("1" if (d == 1 and full[off + i] != 1) else base[off + i] for i, d in enumerate(s)))
    return notas, "".join(base)


# ============================================================================================ rules
class SpmdRule:
    def __init__(self, name, fwd, bwd=None):
        self.name, self._fwd, self._bwd = name, fwd, bwd

    def infer_forward(self, *args, **kwargs):
        return self._fwd(*args, **kwargs)

    def infer_backward(self, *args, **kwargs):
        if self._bwd is None:
            raise NotImplementedError(f"spmd rule {self.name}: no backward rule")
        return self._bwd(*args, **kwargs)


def _matmul_notas(xs, ys, trans_x, trans_y):
    xn, yn = len(xs), len(ys)
    nb = max(xn, yn) - 2
    batch = _letters(max(nb, 0), "mkn")
    xb = xn - 2 if xn >= 2 else 0
    yb = yn - 2 if yn >= 2 else 0

    def batch_part(shape, k):
        out = ""
        for i in range(k):
            letter = batch[nb - k + i]
            out += "1" if shape[i] == 1 and nb > 0 else letter
        return out

    x_nota = batch_part(xs, xb) + ("km" if trans_x else "mk") if xn >= 2 else "k"
    y_nota = batch_part(ys, yb) + ("nk" if trans_y else "kn") if yn >= 2 else "k"
    out = "".join(batch) + ("m" if xn >= 2 else "") + ("n" if yn >= 2 else "")
    return x_nota, y_nota, out


def matmul_forward(x, y, trans_x=False, trans_y=False):
    xn, yn, on = _matmul_notas(x.shape, y.shape, trans_x, trans_y)
    amap = merge_axes([xn, yn], [x.dims_mapping, y.dims_mapping])
    mesh = _mesh([x, y])
    out = _attr(_map(on, amap), mesh, _partial(amap, on))
    return [_attr(_map(xn, amap), mesh), _attr(_map(yn, amap), mesh)], [out]


def matmul_backward(x, y, out, trans_x=False, trans_y=False):
    xn, yn, on = _matmul_notas(x.shape, y.shape, trans_x, trans_y)
    # the output's sharding drives; inputs keep their contracted-axis sharding where compatible
    amap = merge_axes([on, xn, yn], [out.dims_mapping, x.dims_mapping, y.dims_mapping])
    mesh = _mesh([x, y, out])
    return ([_attr(_map(xn, amap), mesh), _attr(_map(yn, amap), mesh)],
            [_attr(_map(on, amap), mesh, _partial(amap, on))])


def elementwise_forward(*xs):
    notas, on = _bcast_notations([x.shape for x in xs])
    amap = merge_axes(notas, [x.dims_mapping for x in xs])
    mesh = _mesh(xs)
    return [_attr(_map(n, amap), mesh) for n in notas], [_attr(_map(on, amap), mesh)]


def elementwise_backward(*specs):
    *xs, out = specs
    notas, on = _bcast_notations([x.shape for x in xs])
    amap = merge_axes([on], [out.dims_mapping])
    mesh = _mesh(specs)
    ins = [_attr(_map(n, amap), mesh) for n in notas]
    # gradient of a broadcast input: summed over the broadcast axes -> partial where those axes were sharded
    grads = [_attr(_map(n, amap), mesh, {amap[a] for a in on if a not in n and amap.get(a, -1) != -1})
             for n in notas]
    return ins, [_attr(_map(on, amap), mesh)] + grads


def reduction_forward(x, axis=None, keepdim=False, reduce_type="sum"):
    nd = len(x.shape)
    axes = list(range(nd)) if axis is None or axis == [] else [a % nd for a in
                                                                 ([axis] if isinstance(axis, int) else axis)]
    xn = "".join(_letters(nd))
    on = "".join(("1" if keepdim else "") if i in axes else xn[i] for i in range(nd))
    amap = merge_axes([xn], [x.dims_mapping])
    mesh = _mesh([x])
    partial = {amap[xn[a]] for a in axes if amap[xn[a]] != -1} if reduce_type in ("sum", "mean") else set()
    if reduce_type not in ("sum", "mean"):  # max / min / prod: cannot be partial -> replicate the reduced axes
        for a in axes:
            amap[xn[a]] = -1
    return [_attr(_map(xn, amap), mesh)], [_attr(_map(on, amap), mesh, partial)]


def _replicate_axes(x, axes):
    nd = len(x.shape)
    dm = list(x.dims_mapping)
    for a in axes:
        dm[a % nd] = -1
    return dm


def softmax_forward(x, axis=-1):
    dm = _replicate_axes(x, [axis])
    mesh = _mesh([x])
    return [_attr(dm, mesh)], [_attr(dm, mesh)]


def softmax_backward(x, out, out_grad, axis=-1):
    dm = _replicate_axes(out_grad, [axis])
    mesh = _mesh([x, out, out_grad])
    return [_attr(dm, mesh), _attr(dm, mesh), _attr(dm, mesh)], [_attr(dm, mesh)]


def layer_norm_forward(x, scale=None, bias=None, epsilon=1e-5, begin_norm_axis=1):
    nd = len(x.shape)
    dm = _replicate_axes(x, range(begin_norm_axis, nd))
    mesh = _mesh([x])
    stat = dm[:begin_norm_axis]
    ins = [_attr(dm, mesh)] + [_attr([-1] * len(s.shape), mesh) for s in (scale, bias) if s is not None]
    return ins, [_attr(dm, mesh), _attr(stat, mesh), _attr(stat, mesh)]


def embedding_forward(ids, weight, padding_idx=-1, sparse=False):
    """weight [V, H]: vocab-sharded weight -> output PARTIAL on that mesh dim (the c_embedding form); hidden-
    sharded weight -> output sharded on its last axis; ids sharding -> output leading axes."""
    mesh = _mesh([ids, weight])
    vd, hd = weight.dims_mapping
    idm = list(ids.dims_mapping)
    used = {m for m in idm if m != -1}
    if hd in used:
        hd = -1
    if vd in used or vd == hd:
        vd = -1
    out = _attr(idm + [hd], mesh, {vd} if vd != -1 else set())
    return [_attr(idm, mesh), _attr([vd, hd], mesh)], [out]


def transpose_forward(x, perm):
    mesh = _mesh([x])
    dm = x.dims_mapping
    return [_attr(dm, mesh)], [_attr([dm[p] for p in perm], mesh)]


def transpose_backward(x, out, perm):
    inv = [0] * len(perm)
    for i, p in enumerate(perm):
        inv[p] = i
    mesh = _mesh([x, out])
    return [_attr([out.dims_mapping[inv[i]] for i in range(len(perm))], mesh)], [_attr(out.dims_mapping, mesh)]


def reshape_forward(x, shape):
    """Maps each output axis to the input axes it is built from; an output axis made by MERGING input axes
    keeps the sharding of the first (outermost) one if it divides, the rest are replicated; a SPLIT input
    axis gives its sharding to the first output piece."""
    src = list(x.shape)
    tot = 1
    for s in src:
        tot *= s
    dst = list(shape)
    if -1 in dst:
        known = 1
        for s in dst:
            known *= s if s != -1 else 1
        dst[dst.index(-1)] = tot // known
    dst = [src[i] if s == 0 else s for i, s in enumerate(dst)]
    mesh = _mesh([x])
    mesh_shape = getattr(mesh, "shape", None)
    in_dm = list(x.dims_mapping)
    out_dm = [-1] * len(dst)
    i = j = 0
    while i < len(src) and j < len(dst):
        gi, gj = [i], [j]
        pi, pj = src[i], dst[j]
        while pi != pj:
            if pi < pj:
                i += 1
                gi.append(i)
                pi *= src[i]
            else:
                j += 1
                gj.append(j)
                pj *= dst[j]
        # size-1 axes never carry a sharding: the group's lead axes are its first non-trivial ones
        si = next((k for k in gi if src[k] != 1), gi[0])
        sj = next((k for k in gj if dst[k] != 1), gj[0])
        lead = in_dm[si]
        for k in gi:
            if k != si:
                in_dm[k] = -1  # only the outermost merged axis keeps a sharding
        if lead != -1:
            n = mesh_shape[lead] if mesh_shape is not None else 1
            if dst[sj] % max(n, 1) == 0:
                out_dm[sj] = lead
            else:
                in_dm[si] = -1
        i, j = i + 1, j + 1
    return [_attr(in_dm, mesh)], [_attr(out_dm, mesh)]


def split_forward(x, num_or_sections, axis=0):
    dm = _replicate_axes(x, [axis])
    mesh = _mesh([x])
    n = num_or_sections if isinstance(num_or_sections, int) else len(num_or_sections)
    return [_attr(dm, mesh)], [_attr(dm, mesh) for _ in range(n)]


def concat_forward(xs, axis=0):
    nd = len(xs[0].shape)
    nota = "".join(_letters(nd))
    amap = merge_axes([nota] * len(xs), [x.dims_mapping for x in xs])
    amap[nota[axis % nd]] = -1
    mesh = _mesh(xs)
    dm = _map(nota, amap)
    return [_attr(dm, mesh) for _ in xs], [_attr(dm, mesh)]


def flash_attention_forward(q, k, v, causal=False):
    """q/k/v [b, s, h, d]: batch and head sharding propagate, sequence and head-dim are replicated (the
    context-parallel split of s is a separate, explicit strategy)."""
    mesh = _mesh([q, k, v])
    amap = merge_axes(["bshd", "bthd", "bthd"], [q.dims_mapping, k.dims_mapping, v.dims_mapping])
    for ax in "std":
        amap[ax] = -1
    qd, kd = _map("bshd", amap), _map("bthd", amap)
    return [_attr(qd, mesh), _attr(kd, mesh), _attr(kd, mesh)], [_attr(qd, mesh), _attr(qd[:1] + [qd[2], -1], mesh)]


def cross_entropy_with_softmax_forward(logits, label, soft_label=False, use_softmax=True, ignore_index=-100,
                                       axis=-1):
    nd = len(logits.shape)
    a = axis % nd
    mesh = _mesh([logits, label])
    nota = "".join(_letters(nd))
    lab_nota = nota[:a] + ("1" if not soft_label else nota[a]) + nota[a + 1:]
    amap = merge_axes([nota, lab_nota], [logits.dims_mapping, label.dims_mapping])
    amap[nota[a]] = -1  # the class axis is replicated (a vocab-sharded head uses c_softmax_with_cross_entropy)
    ld = _map(nota, amap)
    return ([_attr(ld, mesh), _attr(_map(lab_nota, amap), mesh)],
            [_attr(ld, mesh), _attr(_map(lab_nota, amap), mesh)])


def c_softmax_with_cross_entropy_forward(logits, label, ignore_index=-100, rank=0, nranks=1):
    """Vocab-parallel CE: the class axis stays sharded, loss is replicated over it (reduced with allreduce)."""
    mesh = _mesh([logits, label])
    dm = list(logits.dims_mapping)
    return [_attr(dm, mesh), _attr(dm[:-1] + [-1], mesh)], [_attr(dm, mesh), _attr(dm[:-1] + [-1], mesh)]


def default_data_parallel_forward(*xs):
    """Shard the batch axis of every tensor on the mesh dim of the first batch-sharded input."""
    m = next((x.dims_mapping[0] for x in xs if x.dims_mapping and x.dims_mapping[0] != -1), -1)
    mesh = _mesh(xs)
    dms = [[m] + [-1] * (len(x.shape) - 1) if x.shape else [] for x in xs]
    return [_attr(d, mesh) for d in dms], [_attr(dms[0], mesh)]


def replicated_forward(*xs):
    mesh = _mesh(xs)
    return [_attr([-1] * len(x.shape), mesh) for x in xs], [_attr([-1] * len(xs[0].shape), mesh)]


# -------------------------------------------------------------------------------------------- LLM op rules
def _empty(spec):
    return spec is None or not list(getattr(spec, "shape", []) or [])


def rms_norm_forward(x, scale, epsilon=1e-6):
    """Normalisation over the last axis: that axis is replicated, every leading axis keeps its sharding; scale
    is replicated; outputs (y, inverse rms [leading axes])."""
    nd = len(x.shape)
    dm = _replicate_axes(x, [nd - 1])
    mesh = _mesh([x, scale])
    return [_attr(dm, mesh), _attr([-1], mesh)], [_attr(dm, mesh), _attr(dm[:-1], mesh)]


def rms_norm_backward(x, scale, invvar, out_grad, epsilon=1e-6):
    """The output gradient's leading-axis sharding drives; x and out_grad align, d_scale is PARTIAL on the mesh
    dims that shard the leading (summed-over) axes."""
    nd = len(x.shape)
    nota = "".join(_letters(nd))
    amap = merge_axes([nota, nota[:-1], nota], [x.dims_mapping, invvar.dims_mapping, out_grad.dims_mapping])
    amap[nota[-1]] = -1
    mesh = _mesh([x, scale, invvar, out_grad])
    dm = _map(nota, amap)
    return ([_attr(dm, mesh), _attr([-1], mesh), _attr(dm[:-1], mesh), _attr(dm, mesh)],
            [_attr(dm, mesh), _attr([-1], mesh, {m for m in dm[:-1] if m != -1})])


def swiglu_forward(x, y=None):
    """swiglu(x, y) = silu(x) * y: elementwise.  Without y, x = [gate | up] on its last axis: a last-axis
    sharding is accepted as the per-shard [gate_r | up_r] packing of a column-parallel gate_up projection."""
    if _empty(y):
        mesh = _mesh([x])
        return [_attr(x.dims_mapping, mesh), None], [_attr(x.dims_mapping, mesh)]
    return elementwise_forward(x, y)


def swiglu_backward(x, y, out_grad):
    if _empty(y):
        nd = len(x.shape)
        nota = "".join(_letters(nd))
        amap = merge_axes([nota, nota], [out_grad.dims_mapping, x.dims_mapping])
        mesh = _mesh([x, out_grad])
        dm = _map(nota, amap)
        return [_attr(dm, mesh), None, _attr(dm, mesh)], [_attr(dm, mesh), None]
    ins, outs = elementwise_backward(x, y, out_grad)
    return [ins[0], ins[1], outs[0]], outs[1:]


def fused_rope_forward(q, k=None, v=None, sin=None, cos=None, position_ids=None, use_neox_rotary_style=True,
                       time_major=False, rotary_emb_base=10000.0):
    """q/k/v [b, s, h, d] (time_major: [s, b, h, d]) share one notation; head_dim is replicated; the sequence
    axis may stay sharded only when sin/cos are given and position_ids are not (each shard then rotates its own
    positions); a head sharding that does not divide k/v's head count is dropped.  sin/cos follow the
    sequence sharding, position_ids take q's batch / sequence mapping with the sequence replicated."""
    nota = "abcd"
    seq = 0 if time_major else 1
    specs = [q] + [t for t in (k, v) if not _empty(t)]
    notas = [nota] * len(specs)
    dms = [t.dims_mapping for t in specs]
    ids_nota = "ba" if time_major else "ab"
    if not _empty(position_ids):
        notas.append(ids_nota)
        dms.append(position_ids.dims_mapping)
    amap = merge_axes(notas, dms)
    mesh = _mesh(specs)
    dm = _map(nota, amap)
    seq_parallel = not _empty(sin) and not _empty(cos) and _empty(position_ids) and dm[seq] != -1
    dm[3] = -1
    if not seq_parallel:
        dm[seq] = -1
    if dm[2] != -1 and mesh is not None and getattr(mesh, "shape", None) is not None:
        n = mesh.shape[dm[2]]
        for t in specs[1:]:
            if t.shape[2] != q.shape[2] and t.shape[2] % n:
                dm[2] = -1
    qa = _attr(dm, mesh)
    ka = _attr(dm, mesh) if not _empty(k) else None
    va = _attr(dm, mesh) if not _empty(v) else None
    sc = None
    if not _empty(sin):
        snd = len(sin.shape)
        sdm = [-1] * snd
        if seq_parallel:
            sdm[0 if snd == 2 else 1] = dm[seq]
        sc = _attr(sdm, mesh)
    pa = None
    if not _empty(position_ids):
        pdm = _map(ids_nota, amap)
        pdm[1] = -1
        pa = _attr(pdm, mesh)
    return [qa, ka, va, sc, sc, pa], [qa, ka, va]


def c_embedding_forward(weight, x, start_index=0, vocab_size=-1):
    """Vocab-parallel embedding: weight [V, H] rows sharded -> output PARTIAL on that mesh dim (rows outside a
    shard's vocab range contribute zero); ids keep their sharding and give the output's leading axes."""
    nx = len(x.shape)
    xn = "".join(_letters(nx, "jk"))
    amap = merge_axes([xn, "jk"], [x.dims_mapping, weight.dims_mapping])
    mesh = _mesh([weight, x])
    row = weight.dims_mapping[0]
    out = _attr(_map(xn + "k", amap), mesh, {row} if row > -1 else set())
    return [_attr(_map("jk", amap), mesh), _attr(_map(xn, amap), mesh)], [out]


def c_embedding_backward(weight, x, out_grad, start_index=0, vocab_size=-1):
    """d_weight keeps the weight's row sharding; ids and out_grad align on the leading axes (a batch-sharded
    gradient makes d_weight PARTIAL there, which the optimizer-side reduction resolves)."""
    nx = len(x.shape)
    xn = "".join(_letters(nx, "jk"))
    amap = merge_axes([xn, xn + "k"], [x.dims_mapping, out_grad.dims_mapping])
    amap["k"] = -1
    mesh = _mesh([weight, x, out_grad])
    wdm = [weight.dims_mapping[0], -1]
    xdm = _map(xn, amap)
    return ([_attr(wdm, mesh), _attr(xdm, mesh), _attr(_map(xn + "k", amap), mesh)],
            [_attr(wdm, mesh, {m for m in xdm if m != -1})])


def moe_gate_dispatch_forward(x, gate_logits, k=2, capacity=0, use_pad=True):
    """x [S, H], gate_logits [S, E] -> y [E, C, H] (per-expert capacity slots), combine_weights [S, K],
    scatter_index [K, S], expert_offset [E], expert_id [S, K]; the top-k axis is never sharded."""
    amap = merge_axes(["sh", "se"], [x.dims_mapping, gate_logits.dims_mapping])
    amap["k"] = -1
    amap.setdefault("c", -1)
    mesh = _mesh([x, gate_logits])
    ins = [_attr(_map("sh", amap), mesh), _attr(_map("se", amap), mesh)]
    outs = [_attr(_map(n, amap), mesh) for n in ("esh", "sk", "ks", "e", "sk")]
    return ins, outs


def moe_combine_forward(x, combine_weights, scatter_index):
    """y[s, h] = sum_k x[scatter_index[s, k], h] * combine_weights[s, k]: a sharded k makes y PARTIAL (and then
    h may not be sharded as well)."""
    amap = merge_axes(["sh", "sk", "sk"], [x.dims_mapping, combine_weights.dims_mapping,
                                           scatter_index.dims_mapping])
    kd = amap.get("k", -1)
    if kd != -1:
        amap["h"] = -1
    mesh = _mesh([x, combine_weights, scatter_index])
    ins = [_attr(_map("sh", amap), mesh), _attr(_map("sk", amap), mesh), _attr(_map("sk", amap), mesh)]
    return ins, [_attr(_map("sh", amap), mesh, {kd} if kd != -1 else set())]


_RULES = {
    "matmul": SpmdRule("matmul", matmul_forward, matmul_backward),
    "matmul_v2": SpmdRule("matmul_v2", matmul_forward, matmul_backward),
    "elementwise": SpmdRule("elementwise", elementwise_forward, elementwise_backward),
    "reduction": SpmdRule("reduction", reduction_forward),
    "softmax": SpmdRule("softmax", softmax_forward, softmax_backward),
    "layer_norm": SpmdRule("layer_norm", layer_norm_forward),
    "embedding": SpmdRule("embedding", embedding_forward),
    "lookup_table_v2": SpmdRule("lookup_table_v2", embedding_forward),
    "transpose": SpmdRule("transpose", transpose_forward, transpose_backward),
    "reshape": SpmdRule("reshape", reshape_forward),
    "split": SpmdRule("split", split_forward),
    "concat": SpmdRule("concat", concat_forward),
    "flash_attention": SpmdRule("flash_attention", flash_attention_forward),
    "cross_entropy_with_softmax": SpmdRule("cross_entropy_with_softmax", cross_entropy_with_softmax_forward),
    "c_softmax_with_cross_entropy": SpmdRule("c_softmax_with_cross_entropy", c_softmax_with_cross_entropy_forward),
    "default_data_parallel": SpmdRule("default_data_parallel", default_data_parallel_forward),
    "replicated": SpmdRule("replicated", replicated_forward),
    "rms_norm": SpmdRule("rms_norm", rms_norm_forward, rms_norm_backward),
    "swiglu": SpmdRule("swiglu", swiglu_forward, swiglu_backward),
    "fused_rotary_position_embedding": SpmdRule("fused_rotary_position_embedding", fused_rope_forward),
    "fused_rope": SpmdRule("fused_rope", fused_rope_forward),
    "c_embedding": SpmdRule("c_embedding", c_embedding_forward, c_embedding_backward),
    "moe_gate_dispatch": SpmdRule("moe_gate_dispatch", moe_gate_dispatch_forward),
    "moe_combine": SpmdRule("moe_combine", moe_combine_forward),
}
for _n in ("add", "subtract", "multiply", "divide", "maximum", "minimum", "relu", "gelu", "silu", "cast",
           "scale", "where", "dropout", "fused_dropout_add", "pow", "exp", "sqrt", "tanh", "sigmoid"):
    _RULES[_n] = _RULES["elementwise"]
for _n in ("sum", "mean", "max", "min", "prod", "reduce_sum", "reduce_mean", "reduce_max"):
    _RULES[_n] = SpmdRule(_n, (lambda t: (lambda x, axis=None, keepdim=False:
                                          reduction_forward(x, axis, keepdim, t)))(
        "sum" if "sum" in _n else ("mean" if "mean" in _n else "max")))


def get_spmd_rule(name):
    """Rule for an op name; unknown ops fall back to the replicated rule (as the reference does)."""
    return _RULES.get(name, _RULES["replicated"])


get_phi_spmd_rule = get_spmd_rule
