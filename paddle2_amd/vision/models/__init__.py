from .lenet import LeNet  # noqa: F401
from .resnet import (BasicBlock, BottleneckBlock, ResNet, resnet18, resnet34, resnet50, resnet101,  # noqa: F401
                     resnet152, resnext50_32x4d, wide_resnet50_2)
from .vgg import VGG, AlexNet, MobileNetV2, alexnet, mobilenet_v2, vgg11, vgg13, vgg16, vgg19  # noqa: F401
from .mobile import (DenseNet, MobileNetV1, MobileNetV3Large, MobileNetV3Small, ShuffleNetV2, SqueezeNet,  # noqa: F401
                     densenet121, densenet161, densenet169, densenet201, densenet264, mobilenet_v1,
                     mobilenet_v3_large, mobilenet_v3_small, shufflenet_v2_swish, shufflenet_v2_x0_5,
                     shufflenet_v2_x0_25, shufflenet_v2_x0_33, shufflenet_v2_x1_0, shufflenet_v2_x1_5,
                     shufflenet_v2_x2_0, squeezenet1_0, squeezenet1_1)
from .resnet import (resnext50_64x4d, resnext101_32x4d, resnext101_64x4d, resnext152_32x4d,  # noqa: F401
                     resnext152_64x4d, wide_resnet101_2)
from .inception import GoogLeNet, InceptionV3, googlenet, inception_v3  # noqa: F401
