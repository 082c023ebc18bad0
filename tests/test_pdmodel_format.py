"""Reference-format inference models (static/proto.py, static/pdmodel.py): ProgramDesc protobuf wire bytes,
save_combine .pdiparams records, jit.save -> jit.load round trips through the Paddle-op interpreter.  No
reference-written .pdmodel ships in the reference tree, so bit-compatibility is pinned to framework.proto's
field numbers / wire types and lod_tensor.cc's stream layout, checked byte by byte here."""
import io
import struct
import warnings

import numpy as np
import torch

import paddle2_amd as paddle
from paddle2_amd.static import pdmodel
from paddle2_amd.static import proto as P


def test_wire_bytes_known_encodings():
    assert P.encode({"data_type": 5, "dims": [2, 3]}, "TensorDesc") == b"\x08\x05\x10\x02\x10\x03"
    neg = P.encode({"data_type": 5, "dims": [-1, 4]}, "TensorDesc")
    assert neg == b"\x08\x05\x10" + b"\xff" * 9 + b"\x01" + b"\x10\x04"
    assert P.decode(neg, "TensorDesc") == {"data_type": 5, "dims": [-1, 4]}
    # packed repeated ints decode too (proto3-style writers)
    assert P.decode(b"\x08\x05\x12\x02\x02\x03", "TensorDesc")["dims"] == [2, 3]
    a = P.encode({"name": "axis", "type": P.AT["INT"], "i": -1}, "OpDesc.Attr")
    assert P.decode(a, "OpDesc.Attr")["i"] == -1
    f = P.encode({"name": "epsilon", "type": P.AT["FLOAT"], "f": 1e-5}, "OpDesc.Attr")
    assert abs(P.decode(f, "OpDesc.Attr")["f"] - 1e-5) < 1e-12


def test_lod_tensor_stream_layout():
    buf = io.BytesIO()
    x = np.arange(6, dtype=np.float32).reshape(2, 3)
    P.write_lod_tensor(buf, P.VT["FP32"], [2, 3], x.tobytes())
    b = buf.getvalue()
    assert struct.unpack_from("<I", b, 0)[0] == 0 and struct.unpack_from("<Q", b, 4)[0] == 0
    assert struct.unpack_from("<I", b, 12)[0] == 0
    dsz = struct.unpack_from("<i", b, 16)[0]
    assert b[20:20 + dsz] == b"\x08\x05\x10\x02\x10\x03"
    assert np.frombuffer(b[20 + dsz:], dtype=np.float32).tolist() == x.reshape(-1).tolist()
    buf.seek(0)
    dt, dims, raw, lod = P.read_lod_tensor(buf)
    assert dt == 5 and dims == [2, 3] and lod == []


def _roundtrip(net, spec, x, tmp_path, ops_expected):
    net.eval()
    ref = net(paddle.to_tensor(x))
    path = str(tmp_path / "m")
    paddle.jit.save(net, path, input_spec=spec)
    data = open(path + ".pdmodel", "rb").read()
    assert pdmodel.is_program_desc(data)
    desc = P.decode(data, "ProgramDesc")
    types = [o["type"] for o in desc["blocks"][0]["ops"]]
    assert types[0] == "feed" and types[-1] == "fetch"
    for t in ops_expected:
        assert t in types, (t, types)
    loaded = paddle.jit.load(path)
    out = loaded(paddle.to_tensor(x))
    np.testing.assert_allclose(out.numpy(), ref.numpy(), rtol=1e-5, atol=1e-5)
    # the .pdiparams holds every persistable in sorted-name order
    names = pdmodel.program_param_names(desc)
    params = pdmodel.load_params(path + ".pdiparams", names)
    assert len(params) == len(names) and all(isinstance(v, torch.Tensor) for v in params.values())
    return desc


def test_jit_save_lenet_reference_format(tmp_path):
    paddle.seed(1)
    net = paddle.vision.models.LeNet()
    x = np.random.RandomState(0).randn(2, 1, 28, 28).astype("float32")
    spec = [paddle.static.InputSpec([None, 1, 28, 28], "float32", name="image")]
    desc = _roundtrip(net, spec, x, tmp_path, ["conv2d", "pool2d", "relu", "matmul_v2", "elementwise_add",
                                               "flatten_contiguous_range"])
    feed_var = [v for v in desc["blocks"][0]["vars"] if v["name"] == "image"][0]
    assert feed_var["type"]["lod_tensor"]["tensor"]["dims"][0] == -1


def test_jit_save_mlp_layernorm_softmax(tmp_path):
    paddle.seed(2)
    net = paddle.nn.Sequential(paddle.nn.Linear(6, 16), paddle.nn.GELU(), paddle.nn.LayerNorm(16),
                               paddle.nn.Linear(16, 5), paddle.nn.Softmax())
    x = np.random.RandomState(1).randn(3, 6).astype("float32")
    _roundtrip(net, [paddle.static.InputSpec([3, 6], "float32", name="x")], x, tmp_path,
               ["gelu", "layer_norm", "softmax"])


def test_unmapped_op_falls_back_to_native_format(tmp_path):
    class Odd(paddle.nn.Layer):
        def forward(self, x):
            return paddle.cumsum(x, axis=1)

    path = str(tmp_path / "odd")
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        paddle.jit.save(Odd(), path, input_spec=[paddle.static.InputSpec([2, 3], "float32", name="x")])
    assert any("no Paddle op mapping" in str(m.message) for m in w)
    assert not pdmodel.is_program_desc(open(path + ".pdmodel", "rb").read())
    x = np.ones((2, 3), "float32")
    np.testing.assert_allclose(paddle.jit.load(path)(paddle.to_tensor(x)).numpy(), np.cumsum(x, 1))
