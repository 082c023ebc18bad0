"""SPMD sharding-propagation rules (distributed/auto_parallel/spmd_rules.py) on the cases of the reference's
test/auto_parallel/spmd_rules/test_{matmul,elementwise,reduction,softmax,layer_norm,embedding,transpose,reshape,
split,concat}_rule.py (expected dims_mappings / partial dims taken from those tests' assertions)."""
from paddle2_amd.distributed.auto_parallel.spmd_rules import DistTensorSpec, TensorDistAttr, get_phi_spmd_rule


class _Mesh:
    def __init__(self, shape):
        self.shape = shape


MESH = _Mesh([2, 3])


def spec(shape, dm):
    return DistTensorSpec(shape, TensorDistAttr(dm, MESH))


def fwd(name, *args, **kw):
    ins, outs = get_phi_spmd_rule(name).infer_forward(*args, **kw)
    return [a.dims_mapping for a in ins], [(a.dims_mapping, a._partial_dims()) for a in outs]


def test_matmul_rule_cases():
    x, y = [64, 32], [32, 48]
    assert fwd("matmul", spec(x, [1, 0]), spec(y, [0, -1]), False, False) == ([[1, 0], [0, -1]], [([1, -1], {0})])
    assert fwd("matmul", spec(x, [1, -1]), spec(y, [-1, -1]), False, False) == ([[1, -1], [-1, -1]], [([1, -1], set())])
    assert fwd("matmul", spec(x, [-1, -1]), spec(y, [-1, 0]), False, False) == ([[-1, -1], [-1, 0]], [([-1, 0], set())])
    assert fwd("matmul", spec(x, [1, 0]), spec(y, [-1, -1]), False, False) == ([[1, 0], [0, -1]], [([1, -1], {0})])
    assert fwd("matmul", spec(x, [-1, -1]), spec(y, [1, 0]), False, False) == ([[-1, 1], [1, 0]], [([-1, 0], {1})])
    x4 = [512, 48, 64, 32]
    assert fwd("matmul", spec(x4, [0, 1, -1, -1]), spec(y, [-1, -1]), False, False)[1] == [([0, 1, -1, -1], set())]
    ins, outs = fwd("matmul", spec(x4, [1, -1, -1, 0]), spec(y, [-1, -1]), False, False)
    assert ins[1] == [0, -1] and outs == [([1, -1, -1, -1], {0})]
    # trans_x: x = [.., k, m]
    assert fwd("matmul", spec(x4, [1, -1, -1, 0]), spec(y, [-1, -1]), True, False)[1] == [([1, -1, 0, -1], set())]
    # trans_y: y = [n, k]
    ins, outs = fwd("matmul", spec(x4, [-1, -1, -1, -1]), spec([48, 32], [1, 0]), False, True)
    assert ins == [[-1, -1, -1, 0], [1, 0]] and outs == [([-1, -1, -1, 1], {0})]
    # both transposed: the mesh dim 1 conflict (m and n) keeps m
    ins, outs = fwd("matmul", spec(x4, [-1, -1, 0, 1]), spec([48, 32], [1, 0]), True, True)
    assert ins == [[-1, -1, 0, 1], [-1, 0]] and outs == [([-1, -1, 1, -1], {0})]


def test_elementwise_broadcast_and_conflict():
    ins, outs = fwd("add", spec([64, 36, 48], [0, -1, -1]), spec([48], [-1]))
    assert ins == [[0, -1, -1], [-1]] and outs == [([0, -1, -1], set())]
    ins, outs = fwd("add", spec([64, 36, 48], [0, -1, 1]), spec([64, 36, 48], [-1, 1, 1]))
    # axis c: both say 1; mesh dim 1 then also wanted by axis b (later) -> b replicated
    assert outs[0][0] == [0, -1, 1]
    ins, outs = fwd("multiply", spec([64, 1, 48], [0, -1, -1]), spec([64, 36, 48], [-1, 1, -1]))
    assert ins[0] == [0, -1, -1] and outs == [([0, 1, -1], set())]


def test_reduction_partial_and_keepdim():
    assert fwd("sum", spec([64, 32, 48], [0, -1, 1]), axis=[2], keepdim=False) == \
        ([[0, -1, 1]], [([0, -1], {1})])
    assert fwd("sum", spec([64, 32, 48], [0, -1, 1]), axis=[2], keepdim=True)[1] == [([0, -1, -1], {1})]
    assert fwd("max", spec([64, 32, 48], [0, -1, 1]), axis=[2], keepdim=False)[1] == [([0, -1], set())]
    assert fwd("mean", spec([64, 32], [0, 1]))[1] == [([], {0, 1})]


def test_softmax_layernorm_embedding():
    assert fwd("softmax", spec([8, 16, 32], [0, -1, 1]), axis=-1) == ([[0, -1, -1]], [([0, -1, -1], set())])
    ins, outs = fwd("layer_norm", spec([16, 32, 64], [1, -1, 0]), spec([64], [-1]), spec([64], [-1]),
                    begin_norm_axis=2)
    assert ins[0] == [1, -1, -1] and outs[0][0] == [1, -1, -1] and outs[1][0] == [1, -1]
    # vocab-parallel embedding: output partial over the vocab mesh dim
    assert fwd("embedding", spec([4, 1024], [1, -1]), spec([32000, 4096], [0, -1]))[1] == [([1, -1, -1], {0})]
    # hidden-sharded weight: output last axis sharded
    assert fwd("embedding", spec([4, 1024], [0, -1]), spec([32000, 4096], [-1, 1]))[1] == [([0, -1, 1], set())]


def test_transpose_reshape_split_concat():
    assert fwd("transpose", spec([64, 36, 48], [0, -1, 1]), [1, 2, 0])[1] == [([-1, 1, 0], set())]
    ins, outs = fwd("reshape", spec([6, 12, 48, 24], [0, 1, -1, -1]), [1, 72, 48, 4, 6])
    assert outs[0][0] == [-1, 0, -1, -1, -1] and ins[0] == [0, -1, -1, -1]
    ins, outs = fwd("reshape", spec([6, 12, 48, 24], [-1, -1, 1, -1]), [6, 12, 48, 4, 6])
    assert outs[0][0] == [-1, -1, 1, -1, -1]
    ins, outs = fwd("split", spec([64, 32, 48], [0, 1, -1]), 2, axis=1)
    assert ins == [[0, -1, -1]] and [o[0] for o in outs] == [[0, -1, -1]] * 2
    ins, outs = fwd("concat", [spec([64, 32], [0, -1]), spec([64, 32], [-1, 1])], axis=0)
    assert outs == [([-1, 1], set())]


get_spmd_rule = get_phi_spmd_rule
MESH24 = _Mesh([2, 4])


def _spec(shape, dm):
    return DistTensorSpec(shape, TensorDistAttr(dm, MESH24))


def test_c_embedding_rule_reference_cases():
    """test/auto_parallel/spmd_rules/test_c_embedding_rule.py: data parallel, vocab(row)-parallel, backward."""
    r = get_spmd_rule("c_embedding")
    table, x = _spec([512, 768], [-1, -1]), _spec([4, 1024], [1, -1])
    ins, outs = r.infer_forward(table, x, 0, -1)
    assert [a.dims_mapping for a in ins] == [[-1, -1], [1, -1]] and outs[0].dims_mapping == [1, -1, -1]
    table.set_dims_mapping([1, -1])
    x.set_dims_mapping([-1, -1])
    ins, outs = r.infer_forward(table, x, 0, -1)
    assert [a.dims_mapping for a in ins] == [[1, -1], [-1, -1]]
    assert outs[0].dims_mapping == [-1, -1, -1] and outs[0]._is_partial() and outs[0]._partial_dims() == {1}
    out = _spec([4, 1024, 768], [-1, -1, -1])
    ins, outs = r.infer_backward(table, x, out, 0, -1)
    assert [a.dims_mapping for a in ins] == [[1, -1], [-1, -1], [-1, -1, -1]] and outs[0].dims_mapping == [1, -1]
    x.set_dims_mapping([0, -1])
    out.set_dims_mapping([0, -1, -1])
    ins, outs = r.infer_backward(table, x, out, 0, -1)
    assert [a.dims_mapping for a in ins] == [[1, -1], [0, -1], [0, -1, -1]] and outs[0].dims_mapping == [1, -1]
    assert outs[0]._partial_dims() == {0}   # batch-sharded ids: the table gradient is a partial sum


def test_rms_norm_rule():
    r = get_spmd_rule("rms_norm")
    x, w = _spec([4, 16, 64], [0, 1, 1]), _spec([64], [0])
    ins, outs = r.infer_forward(x, w, 1e-6)
    assert ins[0].dims_mapping == [0, 1, -1] and ins[1].dims_mapping == [-1]
    assert outs[0].dims_mapping == [0, 1, -1] and outs[1].dims_mapping == [0, 1]
    og = _spec([4, 16, 64], [0, -1, -1])
    ins, outs = r.infer_backward(x, w, _spec([4, 16], [0, 1]), og, 1e-6)
    assert outs[0].dims_mapping == [0, 1, -1] and outs[1].dims_mapping == [-1] and outs[1]._partial_dims() == {0, 1}


def test_swiglu_rule():
    r = get_spmd_rule("swiglu")
    ins, outs = r.infer_forward(_spec([8, 32], [0, 1]), None)   # packed [gate | up]: per-shard halves allowed
    assert ins[0].dims_mapping == [0, 1] and outs[0].dims_mapping == [0, 1]
    ins, outs = r.infer_forward(_spec([8, 32], [0, -1]), _spec([8, 32], [-1, 1]))
    assert ins[0].dims_mapping == [0, 1] and ins[1].dims_mapping == [0, 1] and outs[0].dims_mapping == [0, 1]


def test_fused_rope_rule():
    r = get_spmd_rule("fused_rotary_position_embedding")
    q = _spec([2, 64, 8, 32], [0, 1, -1, 1])
    k = _spec([2, 64, 8, 32], [0, -1, 1, -1])
    ins, outs = r.infer_forward(q, k, None, None, None, None)
    # no sin/cos: the sequence axis cannot stay sharded; head_dim never is; heads take the free mesh dim
    assert outs[0].dims_mapping == [0, -1, -1, -1] or outs[0].dims_mapping == [0, -1, 1, -1]
    assert outs[0].dims_mapping[3] == -1 and outs[0].dims_mapping[1] == -1
    sin = _spec([64, 32], [-1, -1])
    q2 = _spec([2, 64, 8, 32], [0, 1, -1, -1])
    ins, outs = r.infer_forward(q2, None, None, sin, sin, None)
    assert outs[0].dims_mapping == [0, 1, -1, -1] and ins[3].dims_mapping == [1, -1]   # sequence parallel
    ids = _spec([2, 64], [0, -1])
    ins, outs = r.infer_forward(q2, None, None, sin, sin, ids)
    assert outs[0].dims_mapping == [0, -1, -1, -1] and ins[5].dims_mapping == [0, -1]


def test_moe_gate_dispatch_and_combine_rules():
    ins, outs = get_spmd_rule("moe_gate_dispatch").infer_forward(_spec([64, 32], [0, -1]), _spec([64, 8], [0, 1]),
                                                                 2, 16, True)
    assert [a.dims_mapping for a in ins] == [[0, -1], [0, 1]]
    assert [a.dims_mapping for a in outs] == [[1, 0, -1], [0, -1], [-1, 0], [1], [0, -1]]
    ins, outs = get_spmd_rule("moe_combine").infer_forward(_spec([64, 32], [-1, -1]), _spec([64, 2], [-1, 1]),
                                                           _spec([64, 2], [-1, 1]))
    assert outs[0].dims_mapping == [-1, -1] and outs[0]._partial_dims() == {1}   # sharded k -> partial
    ins, outs = get_spmd_rule("moe_combine").infer_forward(_spec([64, 32], [0, 1]), _spec([64, 2], [0, -1]),
                                                           _spec([64, 2], [0, -1]))
    assert outs[0].dims_mapping == [0, 1] and not outs[0]._partial_dims()
