from .lenet import LeNet  # noqa: F401
from .resnet import (BasicBlock, BottleneckBlock, ResNet, resnet18, resnet34, resnet50, resnet101,  # noqa: F401
                     resnet152, resnext50_32x4d, wide_resnet50_2)
from .vgg import VGG, AlexNet, MobileNetV2, alexnet, mobilenet_v2, vgg11, vgg13, vgg16, vgg19  # noqa: F401
