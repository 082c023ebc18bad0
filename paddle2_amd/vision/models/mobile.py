"""Mobile / compact vision backbones (reference: python/paddle/vision/models/{mobilenetv1,mobilenetv3,
squeezenet,shufflenetv2,densenet,googlenet}.py): MobileNetV1, MobileNetV3 small/large, SqueezeNet
1.0/1.1, ShuffleNetV2 (x0.25-x2.0, swish variant), DenseNet 121/161/169/201/264.

Random-init only (no network for pretrained weights: ``pretrained=True`` raises).  All convolutions
go through nn.Conv2D (MIOpen), so channels-last + bf16 apply as for ResNet50.
"""
from __future__ import annotations

from ... import nn
from ...tensor import manipulation as M


def _no_pretrained(pretrained):
    if pretrained:
        raise ValueError("pretrained weights are not available offline; build with pretrained=False")


def _cbr(cin, cout, k, s=1, groups=1, act=nn.ReLU, padding=None):
    layers = [nn.Conv2D(cin, cout, k, stride=s, padding=(k - 1) // 2 if padding is None else padding, groups=groups,
                        bias_attr=False), nn.BatchNorm2D(cout)]
    if act is not None:
        layers.append(act())
    return nn.Sequential(*layers)


def _div(v, d=8):
    n = max(d, int(v + d / 2) // d * d)
    return n + d if n < 0.9 * v else n


class _Head(nn.Layer):
    def __init__(self, cin, num_classes, with_pool, hidden=None, act=None, dropout=0.0):
        super().__init__()
        self.with_pool, self.num_classes = with_pool, num_classes
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            if hidden:
                self.fc = nn.Sequential(nn.Linear(cin, hidden), act(), nn.Dropout(dropout), nn.Linear(hidden, num_classes))
            else:
                self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        if self.with_pool:
            x = self.pool(x)
        if self.num_classes > 0:
            x = self.fc(M.flatten(x, 1))
        return x


# ------------------------------------------------------------------------------------ MobileNetV1
class MobileNetV1(nn.Layer):
    _CFG = [(32, 64, 1), (64, 128, 2), (128, 128, 1), (128, 256, 2), (256, 256, 1), (256, 512, 2)] + \
           [(512, 512, 1)] * 5 + [(512, 1024, 2), (1024, 1024, 1)]

    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        c = lambda v: int(v * scale)  # noqa: E731
        layers = [_cbr(3, c(32), 3, 2)]
        for cin, cout, s in self._CFG:
            layers += [_cbr(c(cin), c(cin), 3, s, groups=c(cin)), _cbr(c(cin), c(cout), 1)]
        self.features = nn.Sequential(*layers)
        self.head = _Head(c(1024), num_classes, with_pool)

    def forward(self, x):
        return self.head(self.features(x))


# ------------------------------------------------------------------------------------ MobileNetV3
class _SE(nn.Layer):
    def __init__(self, c, r=4):
        super().__init__()
        self.pool = nn.AdaptiveAvgPool2D(1)
        self.fc1 = nn.Conv2D(c, _div(c // r), 1)
        self.fc2 = nn.Conv2D(_div(c // r), c, 1)
        self.relu, self.hs = nn.ReLU(), nn.Hardsigmoid()

    def forward(self, x):
        return x * self.hs(self.fc2(self.relu(self.fc1(self.pool(x)))))


class _IRB(nn.Layer):
    def __init__(self, cin, exp, cout, k, s, se, act):
        super().__init__()
        self.res = s == 1 and cin == cout
        layers = [] if exp == cin else [_cbr(cin, exp, 1, act=act)]
        layers.append(_cbr(exp, exp, k, s, groups=exp, act=act))
        if se:
            layers.append(_SE(exp))
        layers.append(_cbr(exp, cout, 1, act=None))
        self.block = nn.Sequential(*layers)

    def forward(self, x):
        y = self.block(x)
        return x + y if self.res else y


class MobileNetV3(nn.Layer):
    _SMALL = [(3, 16, 16, True, "RE", 2), (3, 72, 24, False, "RE", 2), (3, 88, 24, False, "RE", 1),
              (5, 96, 40, True, "HS", 2), (5, 240, 40, True, "HS", 1), (5, 240, 40, True, "HS", 1),
              (5, 120, 48, True, "HS", 1), (5, 144, 48, True, "HS", 1), (5, 288, 96, True, "HS", 2),
              (5, 576, 96, True, "HS", 1), (5, 576, 96, True, "HS", 1)]
    _LARGE = [(3, 16, 16, False, "RE", 1), (3, 64, 24, False, "RE", 2), (3, 72, 24, False, "RE", 1),
              (5, 72, 40, True, "RE", 2), (5, 120, 40, True, "RE", 1), (5, 120, 40, True, "RE", 1),
              (3, 240, 80, False, "HS", 2), (3, 200, 80, False, "HS", 1), (3, 184, 80, False, "HS", 1),
              (3, 184, 80, False, "HS", 1), (3, 480, 112, True, "HS", 1), (3, 672, 112, True, "HS", 1),
              (5, 672, 160, True, "HS", 2), (5, 960, 160, True, "HS", 1), (5, 960, 160, True, "HS", 1)]

    def __init__(self, config, last_channel, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        c = lambda v: _div(v * scale)  # noqa: E731
        layers = [_cbr(3, c(16), 3, 2, act=nn.Hardswish)]
        cin = c(16)
        for k, exp, cout, se, a, s in config:
            layers.append(_IRB(cin, c(exp), c(cout), k, s, se, nn.ReLU if a == "RE" else nn.Hardswish))
            cin = c(cout)
        last_conv = c(config[-1][1])
        layers.append(_cbr(cin, last_conv, 1, act=nn.Hardswish))
        self.features = nn.Sequential(*layers)
        self.head = _Head(last_conv, num_classes, with_pool, hidden=last_channel, act=nn.Hardswish, dropout=0.2)

    def forward(self, x):
        return self.head(self.features(x))


class MobileNetV3Small(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__(self._SMALL, 1024, scale, num_classes, with_pool)


class MobileNetV3Large(MobileNetV3):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__(self._LARGE, 1280, scale, num_classes, with_pool)


# ------------------------------------------------------------------------------------ SqueezeNet
class _Fire(nn.Layer):
    def __init__(self, cin, sq, e1, e3):
        super().__init__()
        self.sq = nn.Sequential(nn.Conv2D(cin, sq, 1), nn.ReLU())
        self.e1 = nn.Sequential(nn.Conv2D(sq, e1, 1), nn.ReLU())
        self.e3 = nn.Sequential(nn.Conv2D(sq, e3, 3, padding=1), nn.ReLU())

    def forward(self, x):
        x = self.sq(x)
        return M.concat([self.e1(x), self.e3(x)], axis=1)


class SqueezeNet(nn.Layer):
    def __init__(self, version="1.0", num_classes=1000, with_pool=True):
        super().__init__()
        P = lambda: nn.MaxPool2D(3, 2, ceil_mode=True)  # noqa: E731
        if version == "1.0":
            f = [nn.Conv2D(3, 96, 7, stride=2), nn.ReLU(), P(), _Fire(96, 16, 64, 64), _Fire(128, 16, 64, 64),
                 _Fire(128, 32, 128, 128), P(), _Fire(256, 32, 128, 128), _Fire(256, 48, 192, 192),
                 _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), P(), _Fire(512, 64, 256, 256)]
        elif version == "1.1":
            f = [nn.Conv2D(3, 64, 3, stride=2), nn.ReLU(), P(), _Fire(64, 16, 64, 64), _Fire(128, 16, 64, 64), P(),
                 _Fire(128, 32, 128, 128), _Fire(256, 32, 128, 128), P(), _Fire(256, 48, 192, 192),
                 _Fire(384, 48, 192, 192), _Fire(384, 64, 256, 256), _Fire(512, 64, 256, 256)]
        else:
            raise ValueError(f"unsupported SqueezeNet version {version}")
        self.features = nn.Sequential(*f)
        self.num_classes, self.with_pool = num_classes, with_pool
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.5), nn.Conv2D(512, num_classes, 1), nn.ReLU())
        if with_pool:
            self.pool = nn.AdaptiveAvgPool2D(1)

    def forward(self, x):
        x = self.features(x)
        if self.num_classes > 0:
            x = self.classifier(x)
        if self.with_pool:
            x = self.pool(x)
        return M.flatten(x, 1) if self.num_classes > 0 else x


# ------------------------------------------------------------------------------------ ShuffleNetV2
class _Shuffle(nn.Layer):
    def __init__(self, cin, cout, s, act):
        super().__init__()
        self.s = s
        b = cout // 2
        if s > 1:
            self.branch1 = nn.Sequential(_cbr(cin, cin, 3, s, groups=cin, act=None), _cbr(cin, b, 1, act=act))
        bin_ = cin if s > 1 else b
        self.branch2 = nn.Sequential(_cbr(bin_, b, 1, act=act), _cbr(b, b, 3, s, groups=b, act=None),
                                     _cbr(b, b, 1, act=act))
        self.shuffle = nn.ChannelShuffle(2)

    def forward(self, x):
        if self.s == 1:
            x1, x2 = M.split(x, 2, axis=1)
            out = M.concat([x1, self.branch2(x2)], axis=1)
        else:
            out = M.concat([self.branch1(x), self.branch2(x)], axis=1)
        return self.shuffle(out)


class ShuffleNetV2(nn.Layer):
    _CH = {0.25: [24, 24, 48, 96, 512], 0.33: [24, 32, 64, 128, 512], 0.5: [24, 48, 96, 192, 1024],
           1.0: [24, 116, 232, 464, 1024], 1.5: [24, 176, 352, 704, 1024], 2.0: [24, 244, 488, 976, 2048]}

    def __init__(self, scale=1.0, act="relu", num_classes=1000, with_pool=True):
        super().__init__()
        ch = self._CH[scale]
        A = nn.ReLU if act == "relu" else nn.Silu
        layers = [_cbr(3, ch[0], 3, 2, act=A), nn.MaxPool2D(3, 2, padding=1)]
        cin = ch[0]
        for cout, reps in zip(ch[1:4], (4, 8, 4)):
            for i in range(reps):
                layers.append(_Shuffle(cin, cout, 2 if i == 0 else 1, A))
                cin = cout
        layers.append(_cbr(cin, ch[4], 1, act=A))
        self.features = nn.Sequential(*layers)
        self.head = _Head(ch[4], num_classes, with_pool)

    def forward(self, x):
        return self.head(self.features(x))


# ------------------------------------------------------------------------------------ DenseNet
class _DenseLayer(nn.Layer):
    def __init__(self, cin, growth, bn_size, dropout):
        super().__init__()
        self.body = nn.Sequential(nn.BatchNorm2D(cin), nn.ReLU(), nn.Conv2D(cin, bn_size * growth, 1, bias_attr=False),
                                  nn.BatchNorm2D(bn_size * growth), nn.ReLU(),
                                  nn.Conv2D(bn_size * growth, growth, 3, padding=1, bias_attr=False))
        self.drop = nn.Dropout(dropout) if dropout > 0 else None

    def forward(self, x):
        y = self.body(x)
        if self.drop is not None:
            y = self.drop(y)
        return M.concat([x, y], axis=1)


class DenseNet(nn.Layer):
    _CFG = {121: (64, 32, [6, 12, 24, 16]), 161: (96, 48, [6, 12, 36, 24]), 169: (64, 32, [6, 12, 32, 32]),
            201: (64, 32, [6, 12, 48, 32]), 264: (64, 32, [6, 12, 64, 48])}

    def __init__(self, layers=121, bn_size=4, dropout=0.0, num_classes=1000, with_pool=True):
        super().__init__()
        init_c, growth, blocks = self._CFG[layers]
        f = [nn.Conv2D(3, init_c, 7, stride=2, padding=3, bias_attr=False), nn.BatchNorm2D(init_c), nn.ReLU(),
             nn.MaxPool2D(3, 2, padding=1)]
        c = init_c
        for i, n in enumerate(blocks):
            for _ in range(n):
                f.append(_DenseLayer(c, growth, bn_size, dropout))
                c += growth
            if i != len(blocks) - 1:
                f += [nn.BatchNorm2D(c), nn.ReLU(), nn.Conv2D(c, c // 2, 1, bias_attr=False), nn.AvgPool2D(2, 2)]
                c //= 2
        f += [nn.BatchNorm2D(c), nn.ReLU()]
        self.features = nn.Sequential(*f)
        self.head = _Head(c, num_classes, with_pool)

    def forward(self, x):
        return self.head(self.features(x))


def mobilenet_v1(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV1(scale=scale, **kw)


def mobilenet_v3_small(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Small(scale=scale, **kw)


def mobilenet_v3_large(pretrained=False, scale=1.0, **kw):
    _no_pretrained(pretrained)
    return MobileNetV3Large(scale=scale, **kw)


def squeezenet1_0(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return SqueezeNet("1.0", **kw)


def squeezenet1_1(pretrained=False, **kw):
    _no_pretrained(pretrained)
    return SqueezeNet("1.1", **kw)


def _shufflenet(scale, act="relu"):
    def f(pretrained=False, **kw):
        _no_pretrained(pretrained)
        return ShuffleNetV2(scale=scale, act=act, **kw)

    return f


shufflenet_v2_x0_25 = _shufflenet(0.25)
shufflenet_v2_x0_33 = _shufflenet(0.33)
shufflenet_v2_x0_5 = _shufflenet(0.5)
shufflenet_v2_x1_0 = _shufflenet(1.0)
shufflenet_v2_x1_5 = _shufflenet(1.5)
shufflenet_v2_x2_0 = _shufflenet(2.0)
shufflenet_v2_swish = _shufflenet(1.0, "swish")


def _densenet(n):
    def f(pretrained=False, **kw):
        _no_pretrained(pretrained)
        return DenseNet(layers=n, **kw)

    return f


densenet121, densenet161, densenet169, densenet201, densenet264 = (_densenet(n) for n in (121, 161, 169, 201, 264))
