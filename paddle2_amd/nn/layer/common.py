"""Common layers (reference: python/paddle/nn/layer/{common,container,activation,norm,conv,pooling,loss}.py)."""
from __future__ import annotations

import collections

import numpy as np
import torch

from ...framework.param import ParamAttr, Parameter
from ...framework.tensor import Tensor
from .. import functional as F
from .. import initializer as I
from .layers import Layer


# ------------------------------------------------------------------ containers
class Sequential(Layer):
    def __init__(self, *layers):
        super().__init__()
        if len(layers) == 1 and isinstance(layers[0], (list, tuple)) and layers[0] and isinstance(layers[0][0], (list, tuple)):
            layers = layers[0]
        for i, l in enumerate(layers):
            if isinstance(l, (list, tuple)):
                self.add_sublayer(str(l[0]), l[1])
            elif isinstance(l, collections.OrderedDict):
                for k, v in l.items():
                    self.add_sublayer(k, v)
            else:
                self.add_sublayer(str(i), l)

    def __getitem__(self, idx):
        vals = list(self._sub_layers.values())
        if isinstance(idx, slice):
            return Sequential(*vals[idx])
        if isinstance(idx, str):
            return self._sub_layers[idx]
        return vals[idx]

    def __setitem__(self, idx, layer):
        key = list(self._sub_layers.keys())[idx]
        self._sub_layers[key] = layer

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers.values())

    def append(self, layer):
        self.add_sublayer(str(len(self._sub_layers)), layer)
        return self

    def forward(self, x):
        for l in self._sub_layers.values():
            x = l(x)
        return x


class LayerList(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        if sublayers is not None:
            for i, l in enumerate(sublayers):
                self.add_sublayer(str(i), l)

    def __getitem__(self, idx):
        vals = list(self._sub_layers.values())
        if isinstance(idx, slice):
            return LayerList(vals[idx])
        return vals[idx]

    def __setitem__(self, idx, layer):
        if idx < 0:
            idx += len(self)
        self._sub_layers[str(idx)] = layer

    def __delitem__(self, idx):
        vals = list(self._sub_layers.values())
        del vals[idx]
        self._sub_layers.clear()
        for i, l in enumerate(vals):
            self._sub_layers[str(i)] = l

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(list(self._sub_layers.values()))

    def append(self, sublayer):
        self.add_sublayer(str(len(self)), sublayer)
        return self

    def insert(self, index, sublayer):
        vals = list(self._sub_layers.values())
        vals.insert(index, sublayer)
        self._sub_layers.clear()
        for i, l in enumerate(vals):
            self._sub_layers[str(i)] = l

    def extend(self, sublayers):
        for l in sublayers:
            self.append(l)
        return self


ModuleList = LayerList


class LayerDict(Layer):
    def __init__(self, sublayers=None):
        super().__init__()
        if sublayers is not None:
            self.update(sublayers)

    def __getitem__(self, key):
        return self._sub_layers[key]

    def __setitem__(self, key, layer):
        self.add_sublayer(key, layer)

    def __delitem__(self, key):
        del self._sub_layers[key]

    def __len__(self):
        return len(self._sub_layers)

    def __iter__(self):
        return iter(self._sub_layers)

    def __contains__(self, key):
        return key in self._sub_layers

    def keys(self):
        return self._sub_layers.keys()

    def items(self):
        return self._sub_layers.items()

    def values(self):
        return self._sub_layers.values()

    def pop(self, key):
        return self._sub_layers.pop(key)

    def clear(self):
        self._sub_layers.clear()

    def update(self, sublayers):
        items = sublayers.items() if isinstance(sublayers, (dict, collections.OrderedDict, LayerDict)) else sublayers
        for k, v in items:
            self.add_sublayer(k, v)


class ParameterList(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        if parameters is not None:
            for i, p in enumerate(parameters):
                self.add_parameter(str(i), p)

    def __getitem__(self, idx):
        return list(self._parameters.values())[idx]

    def __setitem__(self, idx, p):
        self._parameters[str(idx)] = p

    def __len__(self):
        return len(self._parameters)

    def __iter__(self):
        return iter(list(self._parameters.values()))

    def append(self, p):
        self.add_parameter(str(len(self)), p)
        return self


class ParameterDict(Layer):
    def __init__(self, parameters=None):
        super().__init__()
        if parameters is not None:
            for k, p in parameters.items():
                self.add_parameter(k, p)

    def __getitem__(self, k):
        return self._parameters[k]

    def __setitem__(self, k, p):
        self.add_parameter(k, p)

    def __len__(self):
        return len(self._parameters)

    def keys(self):
        return self._parameters.keys()

    def items(self):
        return self._parameters.items()

    def values(self):
        return self._parameters.values()


# ------------------------------------------------------------------ basic layers
class Identity(Layer):
    def __init__(self, *args, **kwargs):
        super().__init__()

    def forward(self, x):
        return x


class Linear(Layer):
    """y = x @ W + b with W stored [in_features, out_features] (Paddle layout)."""

    def __init__(self, in_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self._in, self._out = in_features, out_features
        self._dtype = self._dtype if self._dtype else "float32"
        from ...framework.dtype import get_default_dtype

        dt = get_default_dtype()
        self.weight = self.create_parameter([in_features, out_features], attr=weight_attr, dtype=dt,
                                            default_initializer=I.XavierUniform())
        battr = ParamAttr._to_attr(bias_attr)
        self.bias = None if battr is False else self.create_parameter([out_features], attr=bias_attr, dtype=dt,
                                                                      is_bias=True)

    def forward(self, x):
        return F.linear(x, self.weight, self.bias)

    def extra_repr(self):
        return f"in_features={self._in}, out_features={self._out}, dtype={self.weight.dtype}"


class Bilinear(Layer):
    def __init__(self, in1_features, in2_features, out_features, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        self.weight = self.create_parameter([out_features, in1_features, in2_features], attr=weight_attr)
        self.bias = self.create_parameter([1, out_features], attr=bias_attr, is_bias=True)

    def forward(self, x1, x2):
        return F.bilinear(x1, x2, self.weight, self.bias)


class Embedding(Layer):
    def __init__(self, num_embeddings, embedding_dim, padding_idx=None, sparse=False, weight_attr=None, name=None):
        super().__init__()
        from ...framework.dtype import get_default_dtype

        self._num, self._dim = num_embeddings, embedding_dim
        self._sparse = sparse
        self._padding_idx = padding_idx if padding_idx is None or padding_idx >= 0 else padding_idx + num_embeddings
        self.weight = self.create_parameter([num_embeddings, embedding_dim], attr=weight_attr,
                                            dtype=get_default_dtype(), default_initializer=I.XavierUniform())
        if self._padding_idx is not None:
            with torch.no_grad():
                self.weight._t[self._padding_idx] = 0

    def forward(self, x):
        return F.embedding(x, self.weight, padding_idx=self._padding_idx, sparse=self._sparse)

    def extra_repr(self):
        return f"{self._num}, {self._dim}"


class Dropout(Layer):
    def __init__(self, p=0.5, axis=None, mode="upscale_in_train", name=None):
        super().__init__()
        self.p, self.axis, self.mode = p, axis, mode

    def forward(self, x):
        return F.dropout(x, self.p, self.axis, self.training, self.mode)

    def extra_repr(self):
        return f"p={self.p}, axis={self.axis}, mode={self.mode}"


class Dropout2D(Layer):
    def __init__(self, p=0.5, data_format="NCHW", name=None):
        super().__init__()
        self.p, self.fmt = p, data_format

    def forward(self, x):
        return F.dropout2d(x, self.p, self.training, self.fmt)


class Dropout3D(Layer):
    def __init__(self, p=0.5, data_format="NCDHW", name=None):
        super().__init__()
        self.p, self.fmt = p, data_format

    def forward(self, x):
        return F.dropout3d(x, self.p, self.training, self.fmt)


class AlphaDropout(Layer):
    def __init__(self, p=0.5, name=None):
        super().__init__()
        self.p = p

    def forward(self, x):
        return F.alpha_dropout(x, self.p, self.training)


class Flatten(Layer):
    def __init__(self, start_axis=1, stop_axis=-1):
        super().__init__()
        self.start_axis, self.stop_axis = start_axis, stop_axis

    def forward(self, x):
        from ...tensor.manipulation import flatten

        return flatten(x, self.start_axis, self.stop_axis)


class Unflatten(Layer):
    def __init__(self, axis, shape, name=None):
        super().__init__()
        self.axis, self.shape = axis, shape

    def forward(self, x):
        from ...tensor.manipulation import unflatten

        return unflatten(x, self.axis, self.shape)


class Pad1D(Layer):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCL", name=None):
        super().__init__()
        self.padding = [padding] * 2 if isinstance(padding, int) else padding
        self.mode, self.value, self.fmt = mode, value, data_format

    def forward(self, x):
        return F.pad(x, self.padding, self.mode, self.value, self.fmt)


class Pad2D(Pad1D):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCHW", name=None):
        super().__init__(padding, mode, value, data_format)
        if isinstance(padding, int):
            self.padding = [padding] * 4


class Pad3D(Pad1D):
    def __init__(self, padding, mode="constant", value=0.0, data_format="NCDHW", name=None):
        super().__init__(padding, mode, value, data_format)
        if isinstance(padding, int):
            self.padding = [padding] * 6


class ZeroPad2D(Pad2D):
    def __init__(self, padding, data_format="NCHW", name=None):
        super().__init__(padding, "constant", 0.0, data_format)


class Upsample(Layer):
    def __init__(self, size=None, scale_factor=None, mode="nearest", align_corners=False, align_mode=0,
                 data_format="NCHW", name=None):
        super().__init__()
        self.size, self.scale_factor, self.mode = size, scale_factor, mode
        self.align_corners, self.fmt = align_corners, data_format

    def forward(self, x):
        return F.interpolate(x, self.size, self.scale_factor, self.mode, self.align_corners, data_format=self.fmt)


class UpsamplingNearest2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format="NCHW", name=None):
        super().__init__(size, scale_factor, "nearest", data_format=data_format)


class UpsamplingBilinear2D(Upsample):
    def __init__(self, size=None, scale_factor=None, data_format="NCHW", name=None):
        super().__init__(size, scale_factor, "bilinear", True, data_format=data_format)


class PixelShuffle(Layer):
    def __init__(self, upscale_factor, data_format="NCHW", name=None):
        super().__init__()
        self.f, self.fmt = upscale_factor, data_format

    def forward(self, x):
        return F.pixel_shuffle(x, self.f, self.fmt)


class PixelUnshuffle(Layer):
    def __init__(self, downscale_factor, data_format="NCHW", name=None):
        super().__init__()
        self.f, self.fmt = downscale_factor, data_format

    def forward(self, x):
        return F.pixel_unshuffle(x, self.f, self.fmt)


class ChannelShuffle(Layer):
    def __init__(self, groups, data_format="NCHW", name=None):
        super().__init__()
        self.g, self.fmt = groups, data_format

    def forward(self, x):
        return F.channel_shuffle(x, self.g, self.fmt)


class CosineSimilarity(Layer):
    def __init__(self, axis=1, eps=1e-8):
        super().__init__()
        self.axis, self.eps = axis, eps

    def forward(self, x1, x2):
        return F.cosine_similarity(x1, x2, self.axis, self.eps)


class PairwiseDistance(Layer):
    def __init__(self, p=2.0, epsilon=1e-6, keepdim=False, name=None):
        super().__init__()
        self.p, self.eps, self.keepdim = p, epsilon, keepdim

    def forward(self, x, y):
        return F.pairwise_distance(x, y, self.p, self.eps, self.keepdim)


class Unfold(Layer):
    def __init__(self, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.k, self.d, self.p, self.s = kernel_sizes, dilations, paddings, strides

    def forward(self, x):
        return F.unfold(x, self.k, self.s, self.p, self.d)


class Fold(Layer):
    def __init__(self, output_sizes, kernel_sizes, dilations=1, paddings=0, strides=1, name=None):
        super().__init__()
        self.o, self.k, self.d, self.p, self.s = output_sizes, kernel_sizes, dilations, paddings, strides

    def forward(self, x):
        return F.fold(x, self.o, self.k, self.s, self.p, self.d)


# ------------------------------------------------------------------ activations
def _act(name, fn, **defaults):
    def __init__(self, *args, name=None, **kwargs):
        Layer.__init__(self)
        keys = list(defaults.keys())
        vals = dict(defaults)
        for k, a in zip(keys, args):
            vals[k] = a
        vals.update({k: v for k, v in kwargs.items() if k in vals})
        self._kw = vals

    def forward(self, x, *extra):  # extra: the indices of the MaxUnPool layers
        return fn(x, *extra, **self._kw)

    def extra_repr(self):
        return ", ".join(f"{k}={v}" for k, v in self._kw.items())

    return type(name, (Layer,), {"__init__": __init__, "forward": forward, "extra_repr": extra_repr})


ReLU = _act("ReLU", F.relu)
ReLU6 = _act("ReLU6", F.relu6)
LeakyReLU = _act("LeakyReLU", F.leaky_relu, negative_slope=0.01)
ELU = _act("ELU", F.elu, alpha=1.0)
CELU = _act("CELU", F.celu, alpha=1.0)
SELU = _act("SELU", F.selu, scale=1.0507009873554804934193349852946, alpha=1.6732632423543772848170429916717)
GELU = _act("GELU", F.gelu, approximate=False)
Silu = _act("Silu", F.silu)
SiLU = Silu
Swish = _act("Swish", F.swish)
Mish = _act("Mish", F.mish)
Sigmoid = _act("Sigmoid", F.sigmoid)
Hardsigmoid = _act("Hardsigmoid", F.hardsigmoid)
Hardswish = _act("Hardswish", F.hardswish)
Hardtanh = _act("Hardtanh", F.hardtanh, min=-1.0, max=1.0)
Hardshrink = _act("Hardshrink", F.hardshrink, threshold=0.5)
Softshrink = _act("Softshrink", F.softshrink, threshold=0.5)
Tanhshrink = _act("Tanhshrink", F.tanhshrink)
ThresholdedReLU = _act("ThresholdedReLU", F.thresholded_relu, threshold=1.0, value=0.0)
Softplus = _act("Softplus", F.softplus, beta=1, threshold=20)
Softsign = _act("Softsign", F.softsign)
Tanh = _act("Tanh", F.tanh)
LogSigmoid = _act("LogSigmoid", F.log_sigmoid)
Softmax = _act("Softmax", F.softmax, axis=-1)
LogSoftmax = _act("LogSoftmax", F.log_softmax, axis=-1)
Maxout = _act("Maxout", F.maxout, groups=2, axis=1)
GLU = _act("GLU", F.glu, axis=-1)
RReLU = _act("RReLU", F.rrelu, lower=1.0 / 8.0, upper=1.0 / 3.0)


class Softmax2D(Layer):
    def forward(self, x):
        return F.softmax(x, axis=-3)


class PReLU(Layer):
    def __init__(self, num_parameters=1, init=0.25, weight_attr=None, data_format="NCHW", name=None):
        super().__init__()
        self.fmt = data_format
        self.weight = self.create_parameter([num_parameters], attr=weight_attr, default_initializer=I.Constant(init))

    def forward(self, x):
        return F.prelu(x, self.weight, self.fmt)


# ------------------------------------------------------------------ conv / pool
class _ConvNd(Layer):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCHW", n=2, transpose=False,
                 output_padding=0):
        super().__init__()
        ks = [kernel_size] * n if isinstance(kernel_size, int) else list(kernel_size)
        self._n, self._transpose = n, transpose
        self._stride, self._padding, self._dilation, self._groups = stride, padding, dilation, groups
        self._data_format, self._padding_mode, self._output_padding = data_format, padding_mode, output_padding
        self._in, self._out = in_channels, out_channels
        if transpose:
            shape = [in_channels, out_channels // groups] + ks
        else:
            shape = [out_channels, in_channels // groups] + ks
        fan_in = (in_channels // groups) * int(np.prod(ks))
        self.weight = self.create_parameter(shape, attr=weight_attr,
                                            default_initializer=I.KaimingUniform(fan_in=fan_in, negative_slope=5 ** 0.5,
                                                                                 nonlinearity="leaky_relu"))
        battr = ParamAttr._to_attr(bias_attr)
        if battr is False:
            self.bias = None
        else:
            bound = 1.0 / np.sqrt(fan_in)
            self.bias = self.create_parameter([out_channels], attr=bias_attr, is_bias=True,
                                              default_initializer=I.Uniform(-bound, bound))

    def extra_repr(self):
        return f"{self._in}, {self._out}, kernel_size={list(self.weight.shape[2:])}, stride={self._stride}, padding={self._padding}"


class Conv1D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format, 1)

    def forward(self, x):
        return F.conv1d(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups, self._data_format)


class Conv2D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format, 2)

    def forward(self, x):
        if self._padding_mode != "zeros":
            p = self._padding if isinstance(self._padding, (list, tuple)) else [self._padding] * 4
            if len(p) == 2:
                p = [p[1], p[1], p[0], p[0]]
            x = F.pad(x, p, mode=self._padding_mode, data_format=self._data_format)
            return F.conv2d(x, self.weight, self.bias, self._stride, 0, self._dilation, self._groups, self._data_format)
        return F.conv2d(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups, self._data_format)


class Conv3D(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, dilation=1, groups=1,
                 padding_mode="zeros", weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, padding_mode,
                         weight_attr, bias_attr, data_format, 3)

    def forward(self, x):
        return F.conv3d(x, self.weight, self.bias, self._stride, self._padding, self._dilation, self._groups, self._data_format)


class Conv1DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, groups=1,
                 dilation=1, weight_attr=None, bias_attr=None, data_format="NCL"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, 1, True, output_padding)

    def forward(self, x, output_size=None):
        return F.conv1d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation, output_size, self._data_format)


class Conv2DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, weight_attr=None, bias_attr=None, data_format="NCHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, 2, True, output_padding)

    def forward(self, x, output_size=None):
        return F.conv2d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._dilation, self._groups, output_size, self._data_format)


class Conv3DTranspose(_ConvNd):
    def __init__(self, in_channels, out_channels, kernel_size, stride=1, padding=0, output_padding=0, dilation=1,
                 groups=1, weight_attr=None, bias_attr=None, data_format="NCDHW"):
        super().__init__(in_channels, out_channels, kernel_size, stride, padding, dilation, groups, "zeros",
                         weight_attr, bias_attr, data_format, 3, True, output_padding)

    def forward(self, x, output_size=None):
        return F.conv3d_transpose(x, self.weight, self.bias, self._stride, self._padding, self._output_padding,
                                  self._groups, self._dilation, output_size, self._data_format)


def _pool_layer(name, fn, argnames):
    def __init__(self, *args, **kwargs):
        Layer.__init__(self)
        kwargs.pop("name", None)
        self._kw = dict(zip(argnames, args))
        self._kw.update(kwargs)

    def forward(self, x, *extra):  # extra: the indices of the MaxUnPool layers
        return fn(x, *extra, **self._kw)

    def extra_repr(self):
        return ", ".join(f"{k}={v}" for k, v in self._kw.items())

    return type(name, (Layer,), {"__init__": __init__, "forward": forward, "extra_repr": extra_repr})


MaxPool1D = _pool_layer("MaxPool1D", F.max_pool1d, ["kernel_size", "stride", "padding", "return_mask", "ceil_mode"])
MaxPool2D = _pool_layer("MaxPool2D", F.max_pool2d, ["kernel_size", "stride", "padding", "return_mask", "ceil_mode", "data_format"])
MaxPool3D = _pool_layer("MaxPool3D", F.max_pool3d, ["kernel_size", "stride", "padding", "return_mask", "ceil_mode", "data_format"])
AvgPool1D = _pool_layer("AvgPool1D", F.avg_pool1d, ["kernel_size", "stride", "padding", "exclusive", "ceil_mode"])
AvgPool2D = _pool_layer("AvgPool2D", F.avg_pool2d, ["kernel_size", "stride", "padding", "ceil_mode", "exclusive", "divisor_override", "data_format"])
AvgPool3D = _pool_layer("AvgPool3D", F.avg_pool3d, ["kernel_size", "stride", "padding", "ceil_mode", "exclusive", "divisor_override", "data_format"])
AdaptiveAvgPool1D = _pool_layer("AdaptiveAvgPool1D", F.adaptive_avg_pool1d, ["output_size"])
AdaptiveAvgPool2D = _pool_layer("AdaptiveAvgPool2D", F.adaptive_avg_pool2d, ["output_size", "data_format"])
AdaptiveAvgPool3D = _pool_layer("AdaptiveAvgPool3D", F.adaptive_avg_pool3d, ["output_size", "data_format"])
AdaptiveMaxPool1D = _pool_layer("AdaptiveMaxPool1D", F.adaptive_max_pool1d, ["output_size", "return_mask"])
AdaptiveMaxPool2D = _pool_layer("AdaptiveMaxPool2D", F.adaptive_max_pool2d, ["output_size", "return_mask"])
AdaptiveMaxPool3D = _pool_layer("AdaptiveMaxPool3D", F.adaptive_max_pool3d, ["output_size", "return_mask"])
MaxUnPool2D = _pool_layer("MaxUnPool2D", F.max_unpool2d, ["kernel_size", "stride", "padding", "data_format", "output_size"])
MaxUnPool1D = _pool_layer("MaxUnPool1D", F.max_unpool1d, ["kernel_size", "stride", "padding", "data_format", "output_size"])
MaxUnPool3D = _pool_layer("MaxUnPool3D", F.max_unpool3d, ["kernel_size", "stride", "padding", "data_format", "output_size"])
LPPool1D = _pool_layer("LPPool1D", F.lp_pool1d, ["norm_type", "kernel_size", "stride", "padding", "ceil_mode", "data_format"])
LPPool2D = _pool_layer("LPPool2D", F.lp_pool2d, ["norm_type", "kernel_size", "stride", "ceil_mode", "data_format"])
FractionalMaxPool2D = _pool_layer("FractionalMaxPool2D", F.fractional_max_pool2d,
                                  ["output_size", "kernel_size", "random_u", "return_mask"])
FractionalMaxPool3D = _pool_layer("FractionalMaxPool3D", F.fractional_max_pool3d,
                                  ["output_size", "kernel_size", "random_u", "return_mask"])


# ------------------------------------------------------------------ norms
class _BatchNormBase(Layer):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCHW", use_global_stats=None, name=None):
        super().__init__()
        self._num_features, self._momentum, self._epsilon = num_features, momentum, epsilon
        self._data_format, self._use_global_stats = data_format, use_global_stats
        if weight_attr is False:
            self.weight = None
        else:
            self.weight = self.create_parameter([num_features], attr=weight_attr, default_initializer=I.Constant(1.0))
        if bias_attr is False:
            self.bias = None
        else:
            self.bias = self.create_parameter([num_features], attr=bias_attr, is_bias=True)
        from ...tensor.creation import ones, zeros

        self.register_buffer("_mean", zeros([num_features]))
        self.register_buffer("_variance", ones([num_features]))

    def forward(self, x, residual=None, act=None):
        """``residual``/``act`` (optional, 'relu') fuse ``act(bn(x) + residual)`` into one kernel."""
        return F.batch_norm(x, self._mean, self._variance, self.weight, self.bias, self.training, self._momentum,
                            self._epsilon, self._data_format, self._use_global_stats, act=act, residual=residual)

    def extra_repr(self):
        return f"num_features={self._num_features}, momentum={self._momentum}, epsilon={self._epsilon}"


class BatchNorm1D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCL", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format, use_global_stats)


class BatchNorm2D(_BatchNormBase):
    pass


class BatchNorm3D(_BatchNormBase):
    def __init__(self, num_features, momentum=0.9, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCDHW", use_global_stats=None, name=None):
        super().__init__(num_features, momentum, epsilon, weight_attr, bias_attr, data_format, use_global_stats)


class BatchNorm(_BatchNormBase):
    def __init__(self, num_channels, act=None, is_test=False, momentum=0.9, epsilon=1e-05, param_attr=None,
                 bias_attr=None, dtype="float32", data_layout="NCHW", in_place=False, moving_mean_name=None,
                 moving_variance_name=None, do_model_average_for_mean_and_var=True, use_global_stats=False,
                 trainable_statistics=False):
        super().__init__(num_channels, momentum, epsilon, param_attr, bias_attr, data_layout, use_global_stats or None)
        self._act = act

    def forward(self, x):
        if self._act in (None, "relu"):
            return super().forward(x, act=self._act)
        return getattr(F, self._act)(super().forward(x))


class SyncBatchNorm(_BatchNormBase):
    """Cross-rank BN: batch statistics all-reduced over the default group (RCCL) in training."""

    def forward(self, x, residual=None, act=None):
        from ...distributed import collective as C

        if not self.training or C.get_world_size() == 1:
            return super().forward(x, residual, act)
        y = self._sync_forward(x)
        if residual is not None:
            y = y + residual
        return F.relu(y) if act == "relu" else y

    def _sync_forward(self, x):
        from ...distributed import collective as C

        t = x._t
        cl = self._data_format in ("NHWC", "NLC", "NDHWC")
        if cl:
            t = t.movedim(-1, 1)
        dims = [0] + list(range(2, t.dim()))
        cnt = torch.tensor([t.numel() / t.shape[1]], device=t.device, dtype=torch.float32)
        s = t.float().sum(dims)
        ss = (t.float() ** 2).sum(dims)
        buf = torch.cat([s, ss, cnt])
        C._all_reduce_torch(buf)
        n = buf[-1]
        mean = buf[: t.shape[1]] / n
        var = buf[t.shape[1]: 2 * t.shape[1]] / n - mean ** 2
        with torch.no_grad():
            self._mean._t.mul_(self._momentum).add_((1 - self._momentum) * mean)
            self._variance._t.mul_(self._momentum).add_((1 - self._momentum) * var * n / (n - 1))
        shp = [1, -1] + [1] * (t.dim() - 2)
        y = (t - mean.reshape(shp).to(t.dtype)) * torch.rsqrt(var.reshape(shp) + self._epsilon).to(t.dtype)
        if self.weight is not None:
            y = y * self.weight._t.reshape(shp) + self.bias._t.reshape(shp)
        if cl:
            y = y.movedim(1, -1)
        return Tensor._wrap(y)

    @classmethod
    def convert_sync_batchnorm(cls, layer):
        if isinstance(layer, _BatchNormBase) and not isinstance(layer, SyncBatchNorm):
            new = SyncBatchNorm(layer._num_features, layer._momentum, layer._epsilon, data_format=layer._data_format)
            new.weight, new.bias = layer.weight, layer.bias
            new._mean, new._variance = layer._mean, layer._variance
            return new
        for k, sub in list(layer._sub_layers.items()):
            layer._sub_layers[k] = cls.convert_sync_batchnorm(sub)
        return layer


class LayerNorm(Layer):
    def __init__(self, normalized_shape, epsilon=1e-05, weight_attr=None, bias_attr=None, name=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = [normalized_shape]
        self._normalized_shape = list(normalized_shape)
        self._epsilon = epsilon
        n = int(np.prod(normalized_shape))
        self.weight = None if weight_attr is False else self.create_parameter(
            self._normalized_shape, attr=weight_attr, default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter(
            self._normalized_shape, attr=bias_attr, is_bias=True)
        self._n = n

    def forward(self, x):
        return F.layer_norm(x, self._normalized_shape, self.weight, self.bias, self._epsilon)

    def extra_repr(self):
        return f"normalized_shape={self._normalized_shape}, epsilon={self._epsilon}"


class RMSNorm(Layer):
    """RMSNorm (paddle.nn.RMSNorm / incubate fused_rms_norm) backed by the HIP kernel."""

    def __init__(self, normalized_shape, epsilon=1e-6, weight_attr=None, name=None):
        super().__init__()
        if isinstance(normalized_shape, int):
            normalized_shape = [normalized_shape]
        self._normalized_shape = list(normalized_shape)
        self._epsilon = epsilon
        from ...framework.dtype import get_default_dtype

        self.weight = self.create_parameter(self._normalized_shape, attr=weight_attr, dtype=get_default_dtype(),
                                            default_initializer=I.Constant(1.0))

    def forward(self, x):
        return F.rms_norm(x, self._normalized_shape, self.weight, self._epsilon)


class GroupNorm(Layer):
    def __init__(self, num_groups, num_channels, epsilon=1e-05, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__()
        self._g, self._eps, self._fmt = num_groups, epsilon, data_format
        self.weight = None if weight_attr is False else self.create_parameter([num_channels], attr=weight_attr,
                                                                               default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_channels], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.group_norm(x, self._g, self._eps, self.weight, self.bias, self._fmt)


class _InstanceNormBase(Layer):
    def __init__(self, num_features, epsilon=1e-05, momentum=0.9, weight_attr=None, bias_attr=None,
                 data_format="NCHW", name=None):
        super().__init__()
        self._eps, self._fmt = epsilon, data_format
        self.scale = None if weight_attr is False else self.create_parameter([num_features], attr=weight_attr,
                                                                              default_initializer=I.Constant(1.0))
        self.bias = None if bias_attr is False else self.create_parameter([num_features], attr=bias_attr, is_bias=True)

    def forward(self, x):
        return F.instance_norm(x, weight=self.scale, bias=self.bias, eps=self._eps, data_format=self._fmt)


InstanceNorm1D = _InstanceNormBase
InstanceNorm2D = _InstanceNormBase
InstanceNorm3D = _InstanceNormBase


class LocalResponseNorm(Layer):
    def __init__(self, size, alpha=0.0001, beta=0.75, k=1.0, data_format="NCHW", name=None):
        super().__init__()
        self.a = (size, alpha, beta, k, data_format)

    def forward(self, x):
        return F.local_response_norm(x, *self.a)


class SpectralNorm(Layer):
    def __init__(self, weight_shape, dim=0, power_iters=1, eps=1e-12, dtype="float32"):
        super().__init__()
        self.dim, self.iters, self.eps = dim, power_iters, eps
        h = weight_shape[dim]
        w = int(np.prod(weight_shape)) // h
        self.weight_u = self.create_parameter([h], default_initializer=I.Normal(0, 1))
        self.weight_v = self.create_parameter([w], default_initializer=I.Normal(0, 1))
        self.weight_u.stop_gradient = True
        self.weight_v.stop_gradient = True

    def forward(self, weight):
        W = weight._t.movedim(self.dim, 0).reshape(weight.shape[self.dim], -1)
        u, v = self.weight_u._t, self.weight_v._t
        with torch.no_grad():
            for _ in range(self.iters):
                v.copy_(torch.nn.functional.normalize(W.t() @ u, dim=0, eps=self.eps))
                u.copy_(torch.nn.functional.normalize(W @ v, dim=0, eps=self.eps))
        sigma = u @ W @ v
        return Tensor._wrap(weight._t / sigma)


# ------------------------------------------------------------------ losses
class _Loss(Layer):
    _fn = None
    _args = ()

    def __init__(self, *args, **kwargs):
        super().__init__()
        kwargs.pop("name", None)
        self._kw = dict(zip(self._args, args))
        self._kw.update(kwargs)

    def forward(self, *inputs):
        return type(self)._fn(*inputs, **self._kw)


def _loss(name, fn, args):
    return type(name, (_Loss,), {"_fn": staticmethod(fn), "_args": tuple(args)})


CrossEntropyLoss = _loss("CrossEntropyLoss", F.cross_entropy,
                         ["weight", "ignore_index", "reduction", "soft_label", "axis", "use_softmax", "label_smoothing"])
MSELoss = _loss("MSELoss", F.mse_loss, ["reduction"])
L1Loss = _loss("L1Loss", F.l1_loss, ["reduction"])
NLLLoss = _loss("NLLLoss", F.nll_loss, ["weight", "ignore_index", "reduction"])
BCELoss = _loss("BCELoss", F.binary_cross_entropy, ["weight", "reduction"])
BCEWithLogitsLoss = _loss("BCEWithLogitsLoss", F.binary_cross_entropy_with_logits, ["weight", "reduction", "pos_weight"])
SmoothL1Loss = _loss("SmoothL1Loss", F.smooth_l1_loss, ["reduction", "delta"])
HuberLoss = _loss("HuberLoss", F.huber_loss, ["reduction", "delta"])
KLDivLoss = _loss("KLDivLoss", F.kl_div, ["reduction", "log_target"])
MarginRankingLoss = _loss("MarginRankingLoss", F.margin_ranking_loss, ["margin", "reduction"])
HingeEmbeddingLoss = _loss("HingeEmbeddingLoss", F.hinge_embedding_loss, ["margin", "reduction"])
CosineEmbeddingLoss = _loss("CosineEmbeddingLoss", F.cosine_embedding_loss, ["margin", "reduction"])
TripletMarginLoss = _loss("TripletMarginLoss", F.triplet_margin_loss, ["margin", "p", "epsilon", "swap", "reduction"])
SoftMarginLoss = _loss("SoftMarginLoss", F.soft_margin_loss, ["reduction"])
MultiLabelSoftMarginLoss = _loss("MultiLabelSoftMarginLoss", F.multi_label_soft_margin_loss, ["weight", "reduction"])
MultiMarginLoss = _loss("MultiMarginLoss", F.multi_margin_loss, ["p", "margin", "weight", "reduction"])
PoissonNLLLoss = _loss("PoissonNLLLoss", F.poisson_nll_loss, ["log_input", "full", "epsilon", "reduction"])
GaussianNLLLoss = _loss("GaussianNLLLoss", F.gaussian_nll_loss, ["full", "epsilon", "reduction"])
CTCLoss = _loss("CTCLoss", F.ctc_loss, ["blank", "reduction"])


class HSigmoidLoss(Layer):
    """Hierarchical sigmoid loss layer (reference nn/layer/loss.py HSigmoidLoss): owns the [num_classes-1,
    feature_size] node weights (or [num_classes, feature_size] with a custom tree) and bias."""

    def __init__(self, feature_size, num_classes, weight_attr=None, bias_attr=None, is_custom=False, is_sparse=False,
                 name=None):
        super().__init__()
        if num_classes < 2 and not is_custom:
            raise ValueError("HSigmoidLoss: num_classes must be >= 2")
        self.num_classes = num_classes
        rows = num_classes if is_custom else num_classes - 1
        self.weight = self.create_parameter([rows, feature_size], attr=weight_attr)
        self.bias = None if bias_attr is False else self.create_parameter([rows, 1], attr=bias_attr, is_bias=True)

    def forward(self, input, label, path_table=None, path_code=None):
        return F.hsigmoid_loss(input, label, self.num_classes, self.weight, self.bias, path_table, path_code)


class RNNTLoss(Layer):
    def __init__(self, blank=0, fastemit_lambda=0.001, reduction="mean", name=None):
        super().__init__()
        self.blank, self.fastemit_lambda, self.reduction = blank, fastemit_lambda, reduction

    def forward(self, input, label, input_lengths, label_lengths):
        return F.rnnt_loss(input, label, input_lengths, label_lengths, self.blank, self.fastemit_lambda, self.reduction)


class CTCLoss(_Loss):  # noqa: F811  (paddle arg order: (log_probs, labels, input_lengths, label_lengths, norm_by_times))
    _args = ("blank", "reduction")

    def forward(self, log_probs, labels, input_lengths, label_lengths, norm_by_times=False):
        return F.ctc_loss(log_probs, labels, input_lengths, label_lengths, **self._kw)
