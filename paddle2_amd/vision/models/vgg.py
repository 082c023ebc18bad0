"""VGG / AlexNet / MobileNetV2 (reference: python/paddle/vision/models/{vgg,alexnet,mobilenetv2}.py)."""
from ... import nn

_CFG = {11: [64, "M", 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        13: [64, 64, "M", 128, 128, "M", 256, 256, "M", 512, 512, "M", 512, 512, "M"],
        16: [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"],
        19: [64, 64, "M", 128, 128, "M", 256, 256, 256, 256, "M", 512, 512, 512, 512, "M", 512, 512, 512, 512, "M"]}


class VGG(nn.Layer):
    def __init__(self, features, num_classes=1000, with_pool=True):
        super().__init__()
        self.features = features
        self.num_classes, self.with_pool = num_classes, with_pool
        if with_pool:
            self.avgpool = nn.AdaptiveAvgPool2D((7, 7))
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Linear(512 * 7 * 7, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, 4096), nn.ReLU(), nn.Dropout(),
                                            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.avgpool(x)
        if self.num_classes > 0:
            x = self.classifier(x.flatten(1))
        return x


def make_layers(cfg, batch_norm=False):
    layers, c = [], 3
    for v in cfg:
        if v == "M":
            layers.append(nn.MaxPool2D(2, 2))
        else:
            layers.append(nn.Conv2D(c, v, 3, padding=1))
            if batch_norm:
                layers.append(nn.BatchNorm2D(v))
            layers.append(nn.ReLU())
            c = v
    return nn.Sequential(*layers)


def vgg11(pretrained=False, batch_norm=False, **kw):
    return VGG(make_layers(_CFG[11], batch_norm), **kw)


def vgg13(pretrained=False, batch_norm=False, **kw):
    return VGG(make_layers(_CFG[13], batch_norm), **kw)


def vgg16(pretrained=False, batch_norm=False, **kw):
    return VGG(make_layers(_CFG[16], batch_norm), **kw)


def vgg19(pretrained=False, batch_norm=False, **kw):
    return VGG(make_layers(_CFG[19], batch_norm), **kw)


class AlexNet(nn.Layer):
    def __init__(self, num_classes=1000):
        super().__init__()
        self.features = nn.Sequential(
            nn.Conv2D(3, 64, 11, stride=4, padding=2), nn.ReLU(), nn.MaxPool2D(3, 2),
            nn.Conv2D(64, 192, 5, padding=2), nn.ReLU(), nn.MaxPool2D(3, 2),
            nn.Conv2D(192, 384, 3, padding=1), nn.ReLU(), nn.Conv2D(384, 256, 3, padding=1), nn.ReLU(),
            nn.Conv2D(256, 256, 3, padding=1), nn.ReLU(), nn.MaxPool2D(3, 2))
        self.avgpool = nn.AdaptiveAvgPool2D((6, 6))
        self.classifier = nn.Sequential(nn.Dropout(), nn.Linear(256 * 36, 4096), nn.ReLU(), nn.Dropout(),
                                        nn.Linear(4096, 4096), nn.ReLU(), nn.Linear(4096, num_classes))

    def forward(self, x):
        return self.classifier(self.avgpool(self.features(x)).flatten(1))


def alexnet(pretrained=False, **kw):
    return AlexNet(**kw)


class _InvRes(nn.Layer):
    def __init__(self, inp, oup, stride, expand):
        super().__init__()
        hid = int(round(inp * expand))
        self.use_res = stride == 1 and inp == oup
        layers = []
        if expand != 1:
            layers += [nn.Conv2D(inp, hid, 1, bias_attr=False), nn.BatchNorm2D(hid), nn.ReLU6()]
        layers += [nn.Conv2D(hid, hid, 3, stride, 1, groups=hid, bias_attr=False), nn.BatchNorm2D(hid), nn.ReLU6(),
                   nn.Conv2D(hid, oup, 1, bias_attr=False), nn.BatchNorm2D(oup)]
        self.conv = nn.Sequential(*layers)

    def forward(self, x):
        return x + self.conv(x) if self.use_res else self.conv(x)


class MobileNetV2(nn.Layer):
    def __init__(self, scale=1.0, num_classes=1000, with_pool=True):
        super().__init__()
        cfg = [[1, 16, 1, 1], [6, 24, 2, 2], [6, 32, 3, 2], [6, 64, 4, 2], [6, 96, 3, 1], [6, 160, 3, 2],
               [6, 320, 1, 1]]
        inp = int(32 * scale)
        last = int(1280 * max(1.0, scale))
        feats = [nn.Conv2D(3, inp, 3, 2, 1, bias_attr=False), nn.BatchNorm2D(inp), nn.ReLU6()]
        for t, c, n, s in cfg:
            oup = int(c * scale)
            for i in range(n):
                feats.append(_InvRes(inp, oup, s if i == 0 else 1, t))
                inp = oup
        feats += [nn.Conv2D(inp, last, 1, bias_attr=False), nn.BatchNorm2D(last), nn.ReLU6()]
        self.features = nn.Sequential(*feats)
        self.with_pool, self.num_classes = with_pool, num_classes
        self.pool2d_avg = nn.AdaptiveAvgPool2D(1)
        if num_classes > 0:
            self.classifier = nn.Sequential(nn.Dropout(0.2), nn.Linear(last, num_classes))

    def forward(self, x):
        x = self.features(x)
        if self.with_pool:
            x = self.pool2d_avg(x)
        if self.num_classes > 0:
            x = self.classifier(x.flatten(1))
        return x


def mobilenet_v2(pretrained=False, scale=1.0, **kw):
    return MobileNetV2(scale, **kw)
