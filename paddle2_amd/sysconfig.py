"""paddle.sysconfig (reference: python/paddle/sysconfig.py): where the framework's headers and native libraries
live, for building custom operators against it (utils.cpp_extension)."""
import os

__all__ = ["get_include", "get_lib"]

_PKG = os.path.dirname(os.path.abspath(__file__))


def get_include():
    """Directory of the framework's C++/HIP headers (csrc/kernels: gemm_core.h, common.h, ...)."""
    src = os.path.join(os.path.dirname(_PKG), "csrc", "kernels")
    return src if os.path.isdir(src) else os.path.join(_PKG, "include")


def get_lib():
    """Directory holding the framework's native libraries (_C, _runtime, the allocator)."""
    return _PKG
