"""paddle.incubate.operators (reference: python/paddle/incubate/operators/): graph sampling / message passing,
the fused softmax-mask kernels and ResNetUnit, re-exported from where the framework implements them."""
from ...geometric import reindex_graph as _reindex_graph
from ...geometric import sample_neighbors as graph_sample_neighbors  # noqa: F401
from ...geometric import send_u_recv as _send_u_recv
from ...ops.extra_ops import graph_khop_sampler  # noqa: F401
from .. import softmax_mask_fuse, softmax_mask_fuse_upper_triangle  # noqa: F401

__all__ = ["graph_send_recv", "graph_khop_sampler", "graph_reindex", "graph_sample_neighbors", "softmax_mask_fuse",
           "softmax_mask_fuse_upper_triangle", "ResNetUnit"]


def graph_send_recv(x, src_index, dst_index, pool_type="sum", out_size=None, name=None):
    return _send_u_recv(x, src_index, dst_index, reduce_op=pool_type.lower(), out_size=out_size)


def graph_reindex(x, neighbors, count, value_buffer=None, index_buffer=None, flag_buffer_hashtable=False,
                  name=None):
    return _reindex_graph(x, neighbors, count, value_buffer, index_buffer)


def __getattr__(name):
    if name == "ResNetUnit":
        return _resnet_unit_cls()
    raise AttributeError(name)


_CLS = []


def _resnet_unit_cls():
    """ResNetUnit layer (reference incubate/operators/resnet_unit.py): conv + BN (+ shortcut conv + BN, or a
    residual add) + ReLU; training uses batch statistics and updates the running ones (NHWC on the MI355X runs
    the native BN kernels through nn.BatchNorm2D)."""
    if _CLS:
        return _CLS[0]
    from ... import nn

    class ResNetUnit(nn.Layer):
        def __init__(self, num_channels_x, num_filters, filter_size, stride=1, momentum=0.9, eps=1e-5,
                     data_format="NHWC", act="relu", fuse_add=False, has_shortcut=False, use_global_stats=False,
                     is_test=False, filter_x_attr=None, scale_x_attr=None, bias_x_attr=None, moving_mean_x_name=None,
                     moving_var_x_name=None, num_channels_z=1, stride_z=1, filter_z_attr=None, scale_z_attr=None,
                     bias_z_attr=None, moving_mean_z_name=None, moving_var_z_name=None):
            super().__init__()
            self._fmt, self._act = data_format, act
            self._fuse_add, self._has_shortcut = fuse_add, has_shortcut
            pad = (filter_size - 1) // 2
            self.conv_x = nn.Conv2D(num_channels_x, num_filters, filter_size, stride, pad, bias_attr=False,
                                    data_format=data_format)
            self.bn_x = nn.BatchNorm2D(num_filters, momentum, eps, data_format=data_format,
                                       use_global_stats=use_global_stats or None)
            if has_shortcut:
                self.conv_z = nn.Conv2D(num_channels_z, num_filters, 1, stride_z, 0, bias_attr=False,
                                        data_format=data_format)
                self.bn_z = nn.BatchNorm2D(num_filters, momentum, eps, data_format=data_format,
                                           use_global_stats=use_global_stats or None)

        def forward(self, x, z=None):
            y = self.bn_x(self.conv_x(x))
            if self._has_shortcut:
                y = y + self.bn_z(self.conv_z(z))
            elif self._fuse_add:
                y = y + z
            return nn.functional.relu(y) if self._act == "relu" else y

    _CLS.append(ResNetUnit)
    return ResNetUnit
