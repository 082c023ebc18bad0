"""Inception-family backbones (reference: python/paddle/vision/models/googlenet.py:130 GoogLeNet,
inceptionv3.py:507 InceptionV3).

GoogLeNet keeps the reference's three-headed output ``(out, aux1, aux2)`` and its bias-free convolutions
with a ReLU after each inception concat; InceptionV3 is the 299x299 Szegedy et al. 2016 network
(stem, 3xA, B, 4xC, D, 2xE) with BN+ReLU convolutions.  Both are random-init (no network for weights).
"""
from __future__ import annotations

import math

from ... import nn
from ...nn import functional as F
from ...tensor import manipulation as M
from .mobile import _cbr, _no_pretrained


class _Conv(nn.Layer):
    """GoogLeNet conv: bias-free, 'same' padding, no norm/activation (the activation follows the concat)."""

    def __init__(self, cin, cout, k, s=1):
        super().__init__()
        self._conv = nn.Conv2D(cin, cout, k, stride=s, padding=(k - 1) // 2, bias_attr=False)

    def forward(self, x):
        return self._conv(x)


class _InceptionV1(nn.Layer):
    def __init__(self, cin, f1, f3r, f3, f5r, f5, proj):
        super().__init__()
        self.b1 = _Conv(cin, f1, 1)
        self.b3 = nn.Sequential(_Conv(cin, f3r, 1), _Conv(f3r, f3, 3))
        self.b5 = nn.Sequential(_Conv(cin, f5r, 1), _Conv(f5r, f5, 5))
        self.pool = nn.MaxPool2D(3, stride=1, padding=1)
        self.proj = _Conv(cin, proj, 1)

    def forward(self, x):
        return F.relu(M.concat([self.b1(x), self.b3(x), self.b5(x), self.proj(self.pool(x))], axis=1))


class GoogLeNet(nn.Layer):
    """Inception v1 with the two auxiliary classifiers; ``forward -> (out, out1, out2)``."""

    _CFG = {"3a": (192, 64, 96, 128, 16, 32, 32), "3b": (256, 128, 128, 192, 32, 96, 64),
            "4a": (480, 192, 96, 208, 16, 48, 64), "4b": (512, 160, 112, 224, 24, 64, 64),
            "4c": (512, 128, 128, 256, 24, 64, 64), "4d": (512, 112, 144, 288, 32, 64, 64),
            "4e": (528, 256, 160, 320, 32, 128, 128), "5a": (832, 256, 160, 320, 32, 128, 128),
            "5b": (832, 384, 192, 384, 48, 128, 128)}

    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.stem = nn.Sequential(_Conv(3, 64, 7, 2), nn.MaxPool2D(3, 2), _Conv(64, 64, 1), _Conv(64, 192, 3))
        self.pool = nn.MaxPool2D(3, 2)
        self.blocks = nn.LayerDict({k: _InceptionV1(*v) for k, v in self._CFG.items()})
        if with_pool:
            self.pool_out = nn.AdaptiveAvgPool2D(1)
            self.pool_aux1 = nn.AvgPool2D(5, stride=3)
            self.pool_aux2 = nn.AvgPool2D(5, stride=3)
        if num_classes > 0:
            self.drop = nn.Dropout(0.4, mode="downscale_in_infer")
            self.fc = nn.Linear(1024, num_classes)
            self.aux1 = nn.Sequential(_Conv(512, 128, 1), nn.Flatten(), nn.Linear(1152, 1024), nn.ReLU(),
                                      nn.Dropout(0.7, mode="downscale_in_infer"), nn.Linear(1024, num_classes))
            # the reference's second auxiliary head has no ReLU between its two Linears (googlenet.py:250)
            self.aux2 = nn.Sequential(_Conv(528, 128, 1), nn.Flatten(), nn.Linear(1152, 1024),
                                      nn.Dropout(0.7, mode="downscale_in_infer"), nn.Linear(1024, num_classes))

    def forward(self, x):
        b = self.blocks
        x = self.pool(self.stem(x))
        x = self.pool(b["3b"](b["3a"](x)))
        a1 = b["4a"](x)
        a2 = b["4d"](b["4c"](b["4b"](a1)))
        x = self.pool(b["4e"](a2))
        out = b["5b"](b["5a"](x))
        if self.with_pool:
            out, a1, a2 = self.pool_out(out), self.pool_aux1(a1), self.pool_aux2(a2)
        if self.num_classes > 0:
            out = self.fc(M.flatten(self.drop(out), 1))
            a1, a2 = self.aux1(a1), self.aux2(a2)
        return out, a1, a2


def googlenet(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return GoogLeNet(**kwargs)


# ------------------------------------------------------------------------------------ InceptionV3
def _c(cin, cout, k, s=1, p=0):
    return _cbr(cin, cout, k, s, padding=p)


class _A(nn.Layer):
    def __init__(self, cin, pool_features):
        super().__init__()
        self.b1 = _c(cin, 64, 1)
        self.b5 = nn.Sequential(_c(cin, 48, 1), _c(48, 64, 5, p=2))
        self.b3 = nn.Sequential(_c(cin, 64, 1), _c(64, 96, 3, p=1), _c(96, 96, 3, p=1))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1, exclusive=False), _c(cin, pool_features, 1))

    def forward(self, x):
        return M.concat([self.b1(x), self.b5(x), self.b3(x), self.bp(x)], axis=1)


class _B(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b3 = _c(cin, 384, 3, 2)
        self.b3d = nn.Sequential(_c(cin, 64, 1), _c(64, 96, 3, p=1), _c(96, 96, 3, 2))
        self.bp = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return M.concat([self.b3(x), self.b3d(x), self.bp(x)], axis=1)


class _C(nn.Layer):
    def __init__(self, cin, c7):
        super().__init__()
        self.b1 = _c(cin, 192, 1)
        self.b7 = nn.Sequential(_c(cin, c7, 1), _c(c7, c7, (1, 7), p=(0, 3)), _c(c7, 192, (7, 1), p=(3, 0)))
        self.b7d = nn.Sequential(_c(cin, c7, 1), _c(c7, c7, (7, 1), p=(3, 0)), _c(c7, c7, (1, 7), p=(0, 3)),
                                 _c(c7, c7, (7, 1), p=(3, 0)), _c(c7, 192, (1, 7), p=(0, 3)))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1, exclusive=False), _c(cin, 192, 1))

    def forward(self, x):
        return M.concat([self.b1(x), self.b7(x), self.b7d(x), self.bp(x)], axis=1)


class _D(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b3 = nn.Sequential(_c(cin, 192, 1), _c(192, 320, 3, 2))
        self.b7 = nn.Sequential(_c(cin, 192, 1), _c(192, 192, (1, 7), p=(0, 3)), _c(192, 192, (7, 1), p=(3, 0)),
                                _c(192, 192, 3, 2))
        self.bp = nn.MaxPool2D(3, 2)

    def forward(self, x):
        return M.concat([self.b3(x), self.b7(x), self.bp(x)], axis=1)


class _E(nn.Layer):
    def __init__(self, cin):
        super().__init__()
        self.b1 = _c(cin, 320, 1)
        self.b3 = _c(cin, 384, 1)
        self.b3a, self.b3b = _c(384, 384, (1, 3), p=(0, 1)), _c(384, 384, (3, 1), p=(1, 0))
        self.b3d = nn.Sequential(_c(cin, 448, 1), _c(448, 384, 3, p=1))
        self.b3da, self.b3db = _c(384, 384, (1, 3), p=(0, 1)), _c(384, 384, (3, 1), p=(1, 0))
        self.bp = nn.Sequential(nn.AvgPool2D(3, 1, 1, exclusive=False), _c(cin, 192, 1))

    def forward(self, x):
        t = self.b3(x)
        d = self.b3d(x)
        return M.concat([self.b1(x), self.b3a(t), self.b3b(t), self.b3da(d), self.b3db(d), self.bp(x)], axis=1)


class InceptionV3(nn.Layer):
    def __init__(self, num_classes=1000, with_pool=True):
        super().__init__()
        self.num_classes, self.with_pool = num_classes, with_pool
        self.stem = nn.Sequential(_c(3, 32, 3, 2), _c(32, 32, 3), _c(32, 64, 3, p=1), nn.MaxPool2D(3, 2),
                                  _c(64, 80, 1), _c(80, 192, 3), nn.MaxPool2D(3, 2))
        blocks = [_A(192, 32), _A(256, 64), _A(288, 64), _B(288)]
        blocks += [_C(768, c7) for c7 in (128, 160, 160, 192)]
        blocks += [_D(768), _E(1280), _E(2048)]
        self.blocks = nn.Sequential(*blocks)
        if with_pool:
            self.avg_pool = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.dropout = nn.Dropout(0.2, mode="downscale_in_infer")
            stdv = 1.0 / math.sqrt(2048.0)
            self.fc = nn.Linear(2048, num_classes, weight_attr=nn.initializer.Uniform(-stdv, stdv))

    def forward(self, x):
        x = self.blocks(self.stem(x))
        if self.with_pool:
            x = self.avg_pool(x)
        if self.num_classes > 0:
            x = self.fc(self.dropout(M.reshape(x, [-1, 2048])))
        return x


def inception_v3(pretrained=False, **kwargs):
    _no_pretrained(pretrained)
    return InceptionV3(**kwargs)
