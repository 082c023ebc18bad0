"""fleet.DistributedStrategy: typed validation, prototxt round trip, degree checks, applied configs
(reference behaviour: python/paddle/distributed/fleet/base/distributed_strategy.py, tests
test/legacy_test/test_fleet_distributed_strategy.py)."""
import pytest

from paddle2_amd.distributed.fleet import DistributedStrategy


def test_defaults_and_types():
    s = DistributedStrategy()
    assert s.amp is False and s.amp_configs["init_loss_scaling"] == 32768.0
    assert s.pipeline_configs["schedule_mode"] == "1F1B"
    assert s.hybrid_configs["sharding_configs"]["comm_buffer_size_MB"] == 256
    s.amp = True
    s.amp_configs = {"init_loss_scaling": 1024, "custom_white_list": ["matmul"]}
    assert s.amp_configs["init_loss_scaling"] == 1024.0 and s.amp_configs["incr_ratio"] == 2.0  # merged
    with pytest.raises(TypeError):
        s.amp = 1
    with pytest.raises(KeyError):
        s.amp_configs = {"init_loss_scale": 2.0}  # typo is rejected, like the proto-backed reference
    with pytest.raises(TypeError):
        s.pipeline_configs = {"accumulate_steps": "4"}
    with pytest.raises(AttributeError):
        s.not_a_field = True
    s.hybrid_configs = {"mp_degree": 2, "pp_configs": {"dp_comm_overlap": True}}
    assert s.hybrid_configs["pp_configs"]["dp_comm_overlap"] and s.hybrid_configs["pp_configs"]["use_batch_p2p_comm"]
    with pytest.raises(KeyError):
        s.hybrid_configs = {"mp_configs": {"no_such": 1}}


def test_prototxt_round_trip(tmp_path):
    s = DistributedStrategy()
    s.recompute = True
    s.recompute_configs = {"checkpoints": ["layers.0", "layers.1"]}
    s.hybrid_configs = {"dp_degree": 2, "mp_degree": 2, "order": ["dp", "sharding", "pp", "sep", "mp"],
                        "sharding_configs": {"comm_buffer_size_MB": 64}}
    s.amp_configs = {"custom_black_list": ["reduce_sum", "exp"], "use_pure_bf16": True}
    f = tmp_path / "strategy.prototxt"
    s.save_to_prototxt(str(f))
    text = f.read_text()
    assert "recompute: true" in text and 'checkpoints: "layers.1"' in text and "hybrid_configs {" in text
    t = DistributedStrategy()
    t.load_from_prototxt(str(f))
    assert t.recompute and t.recompute_configs["checkpoints"] == ["layers.0", "layers.1"]
    assert t.hybrid_configs["dp_degree"] == 2 and t.hybrid_configs["order"][1] == "sharding"
    assert t.hybrid_configs["sharding_configs"]["comm_buffer_size_MB"] == 64
    assert t.amp_configs["custom_black_list"] == ["reduce_sum", "exp"] and t.amp_configs["use_pure_bf16"]
    assert t.to_prototxt() == text


def test_validate_world():
    s = DistributedStrategy()
    s.hybrid_configs = {"mp_degree": 2, "pp_degree": 2}
    assert s.validate_world(8) == 2  # dp filled
    with pytest.raises(ValueError):
        s.validate_world(6)
    s.hybrid_configs = {"dp_degree": 4}
    with pytest.raises(ValueError):
        s.validate_world(8)  # 4*2*2 != 8
    s.hybrid_configs = {"dp_degree": 2, "order": ["dp", "pp", "mp", "mp", "sep"]}
    with pytest.raises(ValueError):
        s.validate_world(8)


def test_fleet_applies_recompute_and_amp():
    import torch

    import paddle2_amd as paddle
    from paddle2_amd.distributed import fleet
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    s = fleet.DistributedStrategy()
    s.recompute = True
    s.amp = True
    s.amp_configs = {"use_pure_bf16": True}
    fleet.init(is_collective=True, strategy=s)
    m = LlamaForCausalLM(LlamaConfig.tiny(dtype="float32"))
    dm = fleet.distributed_model(m)
    assert m.config.recompute  # model-native recompute switched on
    ids = paddle.randint(0, 512, [2, 16])
    from paddle2_amd import amp

    seen = {}
    orig = m.forward

    def spy(*a, **k):
        seen.update(amp.amp_state())
        return orig(*a, **k)

    m.forward = spy
    dm(ids, labels=ids)
    assert seen["enable"] and seen["level"] == "O2" and seen["dtype"] == torch.bfloat16


def test_gradient_merge_in_hybrid_optimizer():
    """gradient_merge k=2 avg: two half-batches merged == one step on the full batch."""
    import torch

    import paddle2_amd as paddle
    from paddle2_amd.distributed import fleet
    from paddle2_amd.distributed.fleet.meta_optimizers import HybridParallelOptimizer

    s = fleet.DistributedStrategy()
    s.gradient_merge = True
    s.gradient_merge_configs = {"k_steps": 2, "avg": True}
    fleet.init(is_collective=True, strategy=s)
    hcg = fleet.get_hybrid_communicate_group()
    torch.manual_seed(0)
    x = torch.randn(8, 4)
    y = torch.randn(8, 3)

    def make():
        paddle.seed(3)
        return paddle.nn.Linear(4, 3)

    a, b = make(), make()
    oa = HybridParallelOptimizer(paddle.optimizer.SGD(0.1, parameters=a.parameters()), hcg, s)
    for half in (slice(0, 4), slice(4, 8)):
        loss = ((a(paddle.to_tensor(x[half])) - paddle.to_tensor(y[half])) ** 2).mean()
        loss.backward()
        oa.step()
        oa.clear_grad()
    ob = paddle.optimizer.SGD(0.1, parameters=b.parameters())
    loss = ((b(paddle.to_tensor(x)) - paddle.to_tensor(y)) ** 2).mean()
    loss.backward()
    ob.step()
    torch.testing.assert_close(a.weight._t, b.weight._t, rtol=1e-5, atol=1e-6)


def test_reference_flags_registered_and_effects():
    import torch

    import paddle2_amd as paddle
    from paddle2_amd.distributed import collective as C
    from paddle2_amd.framework import flags as F
    from paddle2_amd.ops import torch_ops as T

    # every reference flag name is known (paddle/common/flags.cc)
    assert len(F.REFERENCE_FLAGS) == 182
    assert paddle.get_flags("FLAGS_cudnn_exhaustive_search")["FLAGS_cudnn_exhaustive_search"] is False
    # deterministic embedding backward == the atomics path up to fp32 reassociation, bitwise reproducible
    ids = torch.randint(0, 7, (64,))
    w = torch.randn(7, 16, requires_grad=True)
    g = torch.randn(64, 16)
    paddle.set_flags({"FLAGS_embedding_deterministic": 1})
    try:
        outs = []
        for _ in range(2):
            w.grad = None
            T.embedding(ids, w).backward(g)
            outs.append(w.grad.clone())
    finally:
        paddle.set_flags({"FLAGS_embedding_deterministic": 0})
    assert torch.equal(outs[0], outs[1])
    ref = torch.zeros(7, 16).index_add_(0, ids, g)
    torch.testing.assert_close(outs[0], ref)
    # benchmark_nccl records collective timings (world of one: still instrumented)
    paddle.set_flags({"FLAGS_benchmark_nccl": True})
    try:
        C.barrier()
    finally:
        paddle.set_flags({"FLAGS_benchmark_nccl": False})
    assert C.comm_benchmark_stats().get("barrier", [0])[0] >= 1


def test_every_hybrid_subconfig_key_is_classified():
    """honour-or-reject: each mp/pp/sharding sub-key is either implemented or documented as numerically neutral."""
    from paddle2_amd.distributed.fleet.base import distributed_strategy as ds

    for sec, schema in (("mp_configs", ds._MP), ("pp_configs", ds._PP), ("sharding_configs", ds._DYSHARD)):
        table = ds.KEY_SEMANTICS[sec]
        assert set(table) == set(schema), (sec, set(schema) ^ set(table))
        for k, (kind, why) in table.items():
            assert kind in ("honoured", "perf") and why, (sec, k)


def test_sync_param_name_popped_from_mp_configs():
    from paddle2_amd.distributed.fleet import DistributedStrategy

    s = DistributedStrategy()
    assert s.sync_param_name == ["embedding", "layer_norm", ".b_"]
    s.hybrid_configs = {"mp_configs": {"sync_param_name": ["norm"], "sync_grad": True}}
    assert s.sync_param_name == ["norm"] and s.hybrid_configs["mp_configs"]["sync_grad"] is True
