"""Vision model zoo: every constructor builds, runs forward+backward at 64x64 and gives [N, classes]
(reference test strategy: test/legacy_test/test_vision_models.py builds each model and runs a batch)."""
import pytest

import paddle2_amd as paddle
from paddle2_amd.vision import models as M

CASES = ["mobilenet_v1", "mobilenet_v2", "mobilenet_v3_small", "mobilenet_v3_large", "squeezenet1_0", "squeezenet1_1",
         "shufflenet_v2_x0_25", "shufflenet_v2_x1_0", "shufflenet_v2_swish", "densenet121", "resnet18", "alexnet"]


@pytest.mark.parametrize("name", CASES)
def test_model_forward_backward(name):
    paddle.set_device("cpu")
    paddle.seed(0)
    m = getattr(M, name)(num_classes=10)
    size = 224 if name == "alexnet" else 64
    x = paddle.randn([2, 3, size, size])
    y = m(x)
    assert y.shape == [2, 10], y.shape
    y.mean().backward()
    assert any(p.grad is not None for p in m.parameters())


def test_headless_features():
    m = M.mobilenet_v3_small(num_classes=0, with_pool=True)
    y = m(paddle.randn([1, 3, 64, 64]))
    assert y.shape[:2] == [1, 576]
    with pytest.raises(ValueError):
        M.densenet121(pretrained=True)


def test_googlenet_three_heads():
    paddle.seed(0)
    m = M.googlenet(num_classes=7)
    out, a1, a2 = m(paddle.randn([2, 3, 224, 224]))
    assert out.shape == a1.shape == a2.shape == [2, 7]
    (out.mean() + a1.mean() + a2.mean()).backward()
    assert m.aux2[0]._conv.weight.grad is not None


def test_inception_v3_shape_and_size():
    paddle.seed(0)
    m = M.inception_v3(num_classes=5)
    assert m(paddle.randn([1, 3, 299, 299])).shape == [1, 5]
    # same parameter count as the reference InceptionV3 head-less trunk + 2048xC fc
    assert int(sum(p.numel() for p in M.inception_v3().parameters())) == 23834568


@pytest.mark.parametrize("name", ["resnext50_64x4d", "resnext101_32x4d", "wide_resnet101_2"])
def test_resnet_variants_build(name):
    m = getattr(M, name)(num_classes=3)
    assert m(paddle.randn([2, 3, 64, 64])).shape == [2, 3]
