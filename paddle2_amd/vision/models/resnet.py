"""ResNet family (reference: python/paddle/vision/models/resnet.py:228 ResNet, :488 resnet50).

NCHW by default; ``data_format="NHWC"`` keeps activations channels-last, which is the layout
MIOpen's fastest bf16 convolutions want on the MI355X.
"""
from ... import nn
from ...nn.layer.common import _BatchNormBase


def _bn_relu(bn, x, residual=None):
    """relu(bn(x) [+ residual]); one fused HIP kernel for the built-in BatchNorm layers."""
    if isinstance(bn, _BatchNormBase):
        return bn(x, residual=residual, act="relu")
    y = bn(x)
    return nn.functional.relu(y if residual is None else y + residual)


class BasicBlock(nn.Layer):
    expansion = 1

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        self.conv1 = nn.Conv2D(inplanes, planes, 3, padding=1, stride=stride, bias_attr=False, data_format=data_format)
        self.bn1 = norm_layer(planes, data_format=data_format)
        self.relu = nn.ReLU()
        self.conv2 = nn.Conv2D(planes, planes, 3, padding=1, bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(planes, data_format=data_format)
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = _bn_relu(self.bn1, self.conv1(x))
        return _bn_relu(self.bn2, self.conv2(out), identity)  # fused BN + add + ReLU


class BottleneckBlock(nn.Layer):
    expansion = 4

    def __init__(self, inplanes, planes, stride=1, downsample=None, groups=1, base_width=64, dilation=1,
                 norm_layer=None, data_format="NCHW"):
        super().__init__()
        norm_layer = norm_layer or nn.BatchNorm2D
        width = int(planes * (base_width / 64.0)) * groups
        self.conv1 = nn.Conv2D(inplanes, width, 1, bias_attr=False, data_format=data_format)
        self.bn1 = norm_layer(width, data_format=data_format)
        self.conv2 = nn.Conv2D(width, width, 3, padding=dilation, stride=stride, groups=groups, dilation=dilation,
                               bias_attr=False, data_format=data_format)
        self.bn2 = norm_layer(width, data_format=data_format)
        self.conv3 = nn.Conv2D(width, planes * self.expansion, 1, bias_attr=False, data_format=data_format)
        self.bn3 = norm_layer(planes * self.expansion, data_format=data_format)
        self.relu = nn.ReLU()
        self.downsample = downsample
        self.stride = stride

    def forward(self, x):
        identity = x if self.downsample is None else self.downsample(x)
        out = _bn_relu(self.bn1, self.conv1(x))
        out = _bn_relu(self.bn2, self.conv2(out))
        return _bn_relu(self.bn3, self.conv3(out), identity)  # fused BN + add + ReLU


class ResNet(nn.Layer):
    def __init__(self, block, depth=50, width=64, num_classes=1000, with_pool=True, groups=1, data_format="NCHW"):
        super().__init__()
        layer_cfg = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3], 152: [3, 8, 36, 3]}
        layers = layer_cfg[depth]
        self.groups, self.base_width = groups, width
        self.num_classes, self.with_pool = num_classes, with_pool
        self.data_format = data_format
        self._norm_layer = nn.BatchNorm2D
        self.inplanes = 64
        self.dilation = 1
        self.conv1 = nn.Conv2D(3, self.inplanes, 7, stride=2, padding=3, bias_attr=False, data_format=data_format)
        self.bn1 = self._norm_layer(self.inplanes, data_format=data_format)
        self.relu = nn.ReLU()
        self.maxpool = nn.MaxPool2D(kernel_size=3, stride=2, padding=1, data_format=data_format)
        self.layer1 = self._make_layer(block, 64, layers[0])
        self.layer2 = self._make_layer(block, 128, layers[1], stride=2)
        self.layer3 = self._make_layer(block, 256, layers[2], stride=2)
        self.layer4 = self._make_layer(block, 512, layers[3], stride=2)
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((1, 1), data_format=data_format)
        if num_classes > 0:
            self.fc = nn.Linear(512 * block.expansion, num_classes)

    def _make_layer(self, block, planes, blocks, stride=1, dilate=False):
        norm_layer = self._norm_layer
        downsample = None
        if stride != 1 or self.inplanes != planes * block.expansion:
            downsample = nn.Sequential(
                nn.Conv2D(self.inplanes, planes * block.expansion, 1, stride=stride, bias_attr=False,
                          data_format=self.data_format),
                norm_layer(planes * block.expansion, data_format=self.data_format))
        layers = [block(self.inplanes, planes, stride, downsample, self.groups, self.base_width, 1, norm_layer,
                        self.data_format)]
        self.inplanes = planes * block.expansion
        for _ in range(1, blocks):
            layers.append(block(self.inplanes, planes, groups=self.groups, base_width=self.base_width,
                                norm_layer=norm_layer, data_format=self.data_format))
        return nn.Sequential(*layers)

    def forward(self, x):
        x = self.maxpool(_bn_relu(self.bn1, self.conv1(x)))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = x.flatten(1)
            x = self.fc(x)
        return x


def _resnet(block, depth, pretrained=False, **kwargs):
    if pretrained:
        raise ValueError("pretrained weights are not available offline")
    return ResNet(block, depth, **kwargs)


def resnet18(pretrained=False, **kwargs):
    return _resnet(BasicBlock, 18, pretrained, **kwargs)


def resnet34(pretrained=False, **kwargs):
    return _resnet(BasicBlock, 34, pretrained, **kwargs)


def resnet50(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, **kwargs)


def resnet101(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, **kwargs)


def resnet152(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 152, pretrained, **kwargs)


def resnext50_32x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, groups=32, width=4, **kwargs)


def wide_resnet50_2(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, width=128, **kwargs)


def resnext50_64x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 50, pretrained, groups=64, width=4, **kwargs)


def resnext101_32x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, groups=32, width=4, **kwargs)


def resnext101_64x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, groups=64, width=4, **kwargs)


def resnext152_32x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 152, pretrained, groups=32, width=4, **kwargs)


def resnext152_64x4d(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 152, pretrained, groups=64, width=4, **kwargs)


def wide_resnet101_2(pretrained=False, **kwargs):
    return _resnet(BottleneckBlock, 101, pretrained, width=128, **kwargs)
