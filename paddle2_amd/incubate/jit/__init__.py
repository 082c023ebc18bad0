"""paddle.incubate.jit (reference: python/paddle/incubate/jit/inference_decorator.py ``inference``).

``@paddle.incubate.jit.inference`` turns a function or a Layer's forward into an inference engine: the first call
per input signature (shapes / dtypes) converts it with ``paddle.jit.to_static`` under ``no_grad`` (and eval mode
for Layers), optionally in reduced precision (``precision_mode`` float16 / bfloat16 runs it under auto_cast O2),
and with ``cache_static_model`` / ``save_model_dir`` saves the converted program with ``paddle.jit.save``; later
calls hit the cached program.  The TensorRT / CINN switches of the reference are accepted and ignored (no such
backends on the MI355X); ``with_trt=True`` raises.
"""
from __future__ import annotations

import functools

__all__ = ["inference"]


class _InferenceEngine:
    def __init__(self, fn, layer, precision_mode, save_model_dir, cache_static_model):
        from ... import jit

        self.fn, self.layer = fn, layer
        self.precision = precision_mode
        self.save_dir = save_model_dir
        self.cache = cache_static_model
        self._static = jit.to_static(fn)
        self._saved = set()

    def __call__(self, *args, **kwargs):
        from ... import amp, no_grad

        if self.layer is not None:
            self.layer.eval()
        with no_grad():
            if self.precision in ("float16", "bfloat16"):
                with amp.auto_cast(level="O2", dtype=self.precision):
                    out = self._static(*args, **kwargs)
            else:
                out = self._static(*args, **kwargs)
        if self.cache and self.save_dir and self.layer is not None:
            key = tuple((tuple(a.shape), str(a.dtype)) for a in args if hasattr(a, "shape"))
            if key not in self._saved:
                from ... import jit, static

                specs = [static.InputSpec(list(a.shape), a.dtype) for a in args if hasattr(a, "shape")]
                jit.save(self.layer, self.save_dir, input_spec=specs)
                self._saved.add(key)
        return out


def inference(function=None, cache_static_model=False, save_model_dir=None, memory_pool_init_size_mb=1000,
              precision_mode="float32", switch_ir_optim=True, switch_ir_debug=False, enable_cinn=False,
              with_trt=False, trt_precision_mode="float32", trt_use_static=False, collect_shape=False,
              enable_new_ir=False, exp_enable_use_cutlass=False, delete_pass_lists=None, skip_prune_program=False):
    if with_trt:
        raise NotImplementedError("TensorRT is not available on the MI355X build")
    if precision_mode not in ("float32", "float16", "bfloat16"):
        raise ValueError(f"precision_mode must be float32 / float16 / bfloat16, got {precision_mode!r}")

    def deco(f):
        from ...nn.layer.layers import Layer

        if isinstance(f, Layer):
            layer = f
            engine = _InferenceEngine(f.forward, layer, precision_mode, save_model_dir, cache_static_model)
            f.forward = engine
            return f
        engine = _InferenceEngine(f, None, precision_mode, save_model_dir, cache_static_model)
        return functools.wraps(f)(engine)

    return deco(function) if function is not None else deco
