"""End-to-end Llama on the MI355X through the native kernels."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def test_tiny_llama_trains_on_gpu():
    import paddle2_amd as paddle
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.set_device("gpu:0")
    paddle.seed(0)
    cfg = LlamaConfig.tiny()
    m = LlamaForCausalLM(cfg)
    opt = paddle.optimizer.AdamW(3e-3, parameters=m.parameters(), multi_precision=True)
    ids = paddle.randint(0, cfg.vocab_size, [4, 128])
    losses = []
    for _ in range(20):
        loss = m(ids, labels=ids)
        loss.backward()
        opt.step()
        opt.clear_grad()
        losses.append(float(loss))
    assert losses[-1] < losses[0] * 0.7, losses


def test_llama_gpu_matches_cpu_reference():
    """Same weights/data: GPU (HIP kernels, bf16) loss within tolerance of CPU fp32 reference loss."""
    import paddle2_amd as paddle
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.set_device("cpu")
    paddle.seed(1)
    cfg = LlamaConfig.tiny(dtype="float32")
    mc = LlamaForCausalLM(cfg)
    ids = paddle.randint(0, cfg.vocab_size, [2, 64])
    lc = float(mc(ids, labels=ids))
    paddle.set_device("gpu:0")
    cfg_g = LlamaConfig.tiny(dtype="bfloat16")
    mg = LlamaForCausalLM(cfg_g)
    mg.set_state_dict(mc.state_dict())
    ids_g = ids.cuda()
    lg = float(mg(ids_g, labels=ids_g))
    assert abs(lg - lc) < 0.05 * abs(lc), (lg, lc)


def test_llama_is_causal():
    """Changing token t must not change logits at positions < t (catches any attention leak)."""
    import paddle2_amd as paddle
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.set_device("gpu:0")
    paddle.seed(3)
    cfg = LlamaConfig.tiny(num_hidden_layers=2)
    m = LlamaForCausalLM(cfg)
    ids = paddle.randint(0, cfg.vocab_size, [1, 256])
    ids2 = ids.clone()
    t = 150
    ids2[0, t] = (int(ids[0, t]) + 7) % cfg.vocab_size
    with paddle.no_grad():
        a = m(ids)._t.float()
        b = m(ids2)._t.float()
    assert torch.allclose(a[:, :t], b[:, :t], atol=1e-3), (a[:, :t] - b[:, :t]).abs().max()
    assert not torch.allclose(a[:, t:], b[:, t:], atol=1e-3)
