"""paddle.utils.cpp_extension — build user HIP/C++ custom ops for gfx950 (hipcc, no CUDA shims)."""
from __future__ import annotations

import importlib.util
import os
import subprocess
import sysconfig


def _hipcc():
    return os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def load(name, sources, extra_cxx_cflags=None, extra_cuda_cflags=None, extra_ldflags=None,
         extra_include_paths=None, build_directory=None, verbose=False):
    """Compile ``sources`` (.hip/.cc/.cpp with a pybind11 module) into ``name`` and import it."""
    import pybind11

    bd = build_directory or os.path.join(os.path.expanduser("~"), ".cache", "paddle2_amd_ext", name)
    os.makedirs(bd, exist_ok=True)
    out = os.path.join(bd, name + (sysconfig.get_config_var("EXT_SUFFIX") or ".so"))
    inc = ["-I", sysconfig.get_paths()["include"], "-I", pybind11.get_include()]
    for p in extra_include_paths or []:
        inc += ["-I", p]
    cmd = [_hipcc(), "-O3", "-std=c++17", "-fPIC", "-shared", "--offload-arch=gfx950"] + inc + \
        list(extra_cxx_cflags or []) + list(extra_cuda_cflags or []) + list(sources) + ["-o", out] + \
        list(extra_ldflags or [])
    if verbose:
        print(" ".join(cmd))
    subprocess.check_call(cmd)
    spec = importlib.util.spec_from_file_location(name, out)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class CppExtension:
    def __init__(self, sources, *args, **kwargs):
        self.sources = sources
        self.kwargs = kwargs


CUDAExtension = CppExtension


def setup(**attr):
    raise NotImplementedError("use paddle2_amd.utils.cpp_extension.load for JIT builds")
