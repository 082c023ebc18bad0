"""paddle.inference: Config / Predictor over saved inference Programs (reference:
paddle/fluid/inference/api/analysis_predictor.cc, python/paddle/inference/__init__.py).

A Predictor loads ``{prefix}.pdmodel`` / ``{prefix}.pdiparams`` (paddle2_amd.static format), keeps
input/output handles, and runs the Program through the static Executor on the MI355X; with
``enable_cuda_graph()`` (or ``Config.enable_use_gpu`` + graph) each input-shape signature is
captured once in a HIP graph and replayed."""
from __future__ import annotations

import numpy as np
import torch

from ..framework.tensor import Tensor


class PrecisionType:
    Float32 = 0
    Half = 1
    Int8 = 2
    Bfloat16 = 3


class PlaceType:
    CPU = 0
    GPU = 1


class Config:
    def __init__(self, model_file=None, params_file=None):
        if model_file is not None and params_file is None and not model_file.endswith(".pdmodel"):
            self._prefix = model_file
        elif model_file is not None:
            self._prefix = model_file[: -len(".pdmodel")] if model_file.endswith(".pdmodel") else model_file
        else:
            self._prefix = None
        self._gpu = torch.cuda.is_available()
        self._device_id = 0
        self._graph = False

    def set_model(self, model_file, params_file=None):
        self.__init__(model_file, params_file)

    def model_dir(self):
        return self._prefix

    def enable_use_gpu(self, memory_pool_init_size_mb=100, device_id=0, precision_mode=PrecisionType.Float32):
        self._gpu = True
        self._device_id = device_id

    def disable_gpu(self):
        self._gpu = False

    def use_gpu(self):
        return self._gpu

    def gpu_device_id(self):
        return self._device_id

    def enable_cuda_graph(self):
        self._graph = True

    # accepted for API compatibility (graph-level passes are not applicable to replayed Programs)
    def switch_ir_optim(self, x=True):
        pass

    def enable_memory_optim(self, x=True):
        pass

    def enable_mkldnn(self):
        pass

    def switch_use_feed_fetch_ops(self, x=False):
        pass

    def set_cpu_math_library_num_threads(self, n):
        torch.set_num_threads(n)

    def disable_glog_info(self):
        pass


class _Handle:
    def __init__(self, name):
        self.name = name
        self._value = None

    def reshape(self, shape):
        self._shape = list(shape)

    def copy_from_cpu(self, arr):
        self._value = np.asarray(arr)

    def share_external_data(self, t):
        self._value = t

    def copy_to_cpu(self):
        v = self._value
        if isinstance(v, Tensor):
            v = v._t
        if isinstance(v, torch.Tensor):
            v = v.detach()
            return (v.float() if v.dtype == torch.bfloat16 else v).cpu().numpy()
        return v

    def shape(self):
        v = self._value
        return list(v.shape) if v is not None else []

    def type(self):
        return getattr(self._value, "dtype", None)


class Predictor:
    def __init__(self, config: Config):
        from ..static import BuildStrategy, CompiledProgram, Executor, load_inference_model

        dev = f"gpu:{config._device_id}" if (config._gpu and torch.cuda.is_available()) else "cpu"
        from ..framework.place import _parse_device

        self._exe = Executor(_parse_device(dev))
        prog, feeds, fetch = load_inference_model(config._prefix, self._exe)
        self._feeds, self._fetch = feeds, fetch
        if config._graph and dev != "cpu":
            bs = BuildStrategy()
            bs.enable_cuda_graph = True
            self._prog = CompiledProgram(prog, bs)
        else:
            self._prog = prog
        self._in = {n: _Handle(n) for n in feeds}
        self._out_names = [f"fetch_{i}" for i in range(len(fetch))]
        self._out = {n: _Handle(n) for n in self._out_names}

    def get_input_names(self):
        return list(self._feeds)

    def get_output_names(self):
        return list(self._out_names)

    def get_input_handle(self, name):
        return self._in[name]

    def get_output_handle(self, name):
        return self._out[name]

    def run(self, inputs=None):
        if inputs is not None:
            for n, v in zip(self._feeds, inputs):
                self._in[n]._value = v
        feed = {n: (h._value._t if isinstance(h._value, Tensor) else h._value) for n, h in self._in.items()}
        res = self._exe.run(self._prog, feed=feed, fetch_list=self._fetch, return_numpy=False)
        for n, r in zip(self._out_names, res):
            self._out[n]._value = r
        if inputs is not None:
            return res
        return True

    def clone(self):
        return self

    def clear_intermediate_tensor(self):
        pass

    def try_shrink_memory(self):
        pass


def create_predictor(config):
    return Predictor(config)


def get_version():
    from ..version import full_version

    return full_version
