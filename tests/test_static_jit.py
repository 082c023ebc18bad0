"""Static Program capture + Executor, jit.to_static/save/load, inference Predictor
(reference tests: test/legacy_test/test_executor_*.py, test_jit_save_load.py, test/dygraph_to_static/*,
test/cpp/inference api tests)."""
import numpy as np
import pytest
import torch

import paddle2_amd as paddle


def _build_mlp():
    main, startup = paddle.static.Program(), paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main, startup):
            x = paddle.static.data("x", [-1, 8], "float32")
            y = paddle.static.data("y", [-1, 1], "int64")
            h = paddle.static.nn.fc(x, 16, activation="relu")
            logits = paddle.static.nn.fc(h, 3)
            loss = paddle.nn.functional.cross_entropy(logits, y)
            opt = paddle.optimizer.SGD(0.5, parameters=main.all_parameters())
            opt.minimize(loss)
    finally:
        paddle.disable_static()
    return main, startup, logits, loss


def test_static_program_trains_and_matches_dygraph():
    paddle.seed(0)
    main, startup, logits, loss = _build_mlp()
    by_shape = {tuple(p.shape): p for p in main.all_parameters()}
    # dygraph twin with identical weights
    w1, b1, w2, b2 = [by_shape[s]._t.detach().clone() for s in [(8, 16), (16,), (16, 3), (3,)]]
    exe = paddle.static.Executor(paddle.CPUPlace())
    exe.run(startup)
    rs = np.random.RandomState(0)
    X = rs.randn(32, 8).astype("float32")
    Y = X[:, :3].argmax(1)[:, None].astype("int64")
    for it in range(3):
        (l,) = exe.run(main, feed={"x": X, "y": Y}, fetch_list=[loss])
        tw = [t.requires_grad_() for t in (w1, b1, w2, b2)]
        h = torch.relu(torch.from_numpy(X) @ tw[0] + tw[1])
        z = h @ tw[2] + tw[3]
        rl = torch.nn.functional.cross_entropy(z, torch.from_numpy(Y[:, 0]))
        rl.backward()
        with torch.no_grad():
            for t in tw:
                t -= 0.5 * t.grad
                t.grad = None
        w1, b1, w2, b2 = [t.detach() for t in tw]
        assert abs(float(l) - float(rl)) < 1e-5


def test_static_append_backward_fetch_grads_and_prune():
    paddle.seed(1)
    main = paddle.static.Program()
    paddle.enable_static()
    try:
        with paddle.static.program_guard(main):
            x = paddle.static.data("x", [4, 3], "float32")
            lin = paddle.nn.Linear(3, 2)
            out = lin(x)
            loss = (out * out).mean()
            pg = paddle.static.append_backward(loss)
    finally:
        paddle.disable_static()
    exe = paddle.static.Executor()
    X = np.ones((4, 3), "float32")
    gvar = [g for p, g in pg if p is lin.weight][0]
    l, gw = exe.run(main, feed={"x": X}, fetch_list=[loss, gvar])
    xt = torch.ones(4, 3)
    w = lin.weight._t.detach().clone().requires_grad_()
    ((xt @ w + lin.bias._t.detach()) ** 2).mean().backward()
    np.testing.assert_allclose(gw, w.grad.numpy(), rtol=1e-5)
    test = main.clone(for_test=True)
    (o,) = exe.run(test, feed={"x": X}, fetch_list=[out])
    assert o.shape == (4, 2)


def test_save_load_inference_model_and_predictor(tmp_path):
    paddle.seed(0)
    main, startup, logits, loss = _build_mlp()
    exe = paddle.static.Executor()
    test = main.clone(for_test=True)
    x = paddle.Tensor._wrap(main.feeds["x"])
    prefix = str(tmp_path / "mlp")
    paddle.static.save_inference_model(prefix, [x], [logits], exe, program=test)
    prog, feeds, fetch = paddle.static.load_inference_model(prefix, exe)
    X = np.random.randn(5, 8).astype("float32")
    (a,) = exe.run(test, feed={"x": X}, fetch_list=[logits])
    (b,) = exe.run(prog, feed={feeds[0]: X}, fetch_list=fetch)
    np.testing.assert_allclose(a, b)
    from paddle2_amd import inference

    pred = inference.create_predictor(inference.Config(prefix))
    pred.get_input_handle(pred.get_input_names()[0]).copy_from_cpu(X)
    pred.run()
    np.testing.assert_allclose(pred.get_output_handle(pred.get_output_names()[0]).copy_to_cpu(), a, rtol=1e-6)


def test_jit_to_static_save_load(tmp_path):
    paddle.seed(0)
    net = paddle.vision.models.LeNet()
    x = paddle.randn([4, 1, 28, 28])
    ref = net(x)
    snet = paddle.jit.to_static(net)
    out = snet(x)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=1e-6)
    out.sum().backward()
    assert net.parameters()[0].grad is not None
    path = str(tmp_path / "lenet")
    paddle.jit.save(net, path, input_spec=[paddle.static.InputSpec([None, 1, 28, 28], "float32")])
    tl = paddle.jit.load(path)
    np.testing.assert_allclose(tl(x).numpy(), ref.numpy(), atol=1e-6)


def test_static_llama_uses_native_op_entries():
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.seed(2)
    m = LlamaForCausalLM(LlamaConfig.tiny(dtype="float32", num_hidden_layers=1))
    ids = paddle.randint(0, 512, [2, 16])
    ref = m(ids)
    sf = paddle.jit.to_static(lambda t: m(t))
    out = sf(ids)
    np.testing.assert_allclose(out.numpy(), ref.numpy(), atol=1e-5)
    names = [o.name for o in sf.concrete_program.ops]
    assert any("qkv_rope_attention" in n for n in names) and any("rms_norm" in n for n in names), names


@pytest.mark.gpu
def test_static_program_hip_graph_gpu():
    from paddle2_amd.models import LlamaConfig, LlamaForCausalLM

    paddle.set_device("gpu:0")
    paddle.seed(2)
    m = LlamaForCausalLM(LlamaConfig.tiny(num_hidden_layers=2))
    m.eval()
    ids = paddle.randint(0, 512, [2, 64])
    with torch.no_grad():
        ref = m(ids)
    bs = paddle.static.BuildStrategy()
    bs.enable_cuda_graph = True
    sf = paddle.jit.to_static(lambda t: m(t), build_strategy=bs)
    with torch.no_grad():
        o1 = sf(ids)
        o2 = sf(ids)  # graph replay
    torch.testing.assert_close(o1._t.float(), ref._t.float(), atol=2e-2, rtol=2e-2)
    torch.testing.assert_close(o2._t.float(), o1._t.float())
