"""Places and the global default device.

Mirrors paddle's Place family (phi/common/place.h) and ``paddle.set_device``/``get_device``
(python/paddle/device/__init__.py). On ROCm the GPU place is still called ``CUDAPlace`` in
Paddle; we keep that spelling for API compatibility, but the only accelerator is an MI355X
(HIP device, torch device type ``"cuda"`` under ROCm).
"""
from __future__ import annotations

import os

import torch


class Place:
    _kind = "undefined"

    def __init__(self, device_id: int = 0):
        self._id = int(device_id)

    def get_device_id(self) -> int:
        return self._id

    def is_gpu_place(self) -> bool:
        return self._kind == "gpu"

    def is_cpu_place(self) -> bool:
        return self._kind == "cpu"

    def is_cuda_pinned_place(self) -> bool:
        return self._kind == "gpu_pinned"

    def torch_device(self) -> torch.device:
        if self._kind == "gpu":
            return torch.device("cuda", self._id)
        return torch.device("cpu")

    def __eq__(self, other):
        return isinstance(other, Place) and self._kind == other._kind and self._id == other._id

    def __hash__(self):
        return hash((self._kind, self._id))


class CPUPlace(Place):
    _kind = "cpu"

    def __init__(self):
        super().__init__(0)

    def __repr__(self):
        return "Place(cpu)"


class CUDAPlace(Place):
    _kind = "gpu"

    def __repr__(self):
        return f"Place(gpu:{self._id})"


class CUDAPinnedPlace(Place):
    _kind = "gpu_pinned"

    def __init__(self):
        super().__init__(0)

    def __repr__(self):
        return "Place(gpu_pinned)"


# Paddle exposes XPUPlace/CustomPlace etc.; they are out of scope on MI355X but we keep
# names so user code that merely references them imports.
class XPUPlace(Place):
    _kind = "xpu"


class CustomPlace(Place):
    _kind = "custom"

    def __init__(self, dev_type="custom", device_id=0):
        super().__init__(device_id)
        self.dev_type = dev_type


IPUPlace = XPUPlace


def _gpu_available() -> bool:
    return torch.cuda.is_available()


def _initial_device() -> torch.device:
    env = os.environ.get("PADDLE2_AMD_DEVICE")
    if env:
        return _parse_device(env)
    if _gpu_available():
        local = int(os.environ.get("LOCAL_RANK", os.environ.get("PADDLE_LOCAL_RANK", "0")))
        n = torch.cuda.device_count()
        return torch.device("cuda", local % max(n, 1))
    return torch.device("cpu")


def _parse_device(device) -> torch.device:
    if isinstance(device, torch.device):
        return device
    if isinstance(device, Place):
        return device.torch_device()
    s = str(device).lower()
    if s in ("cpu",):
        return torch.device("cpu")
    if s.startswith("gpu") or s.startswith("cuda") or s.startswith("hip"):
        idx = 0
        if ":" in s:
            idx = int(s.split(":")[1])
        return torch.device("cuda", idx)
    raise ValueError(f"unsupported device {device!r}")


_current_device: torch.device | None = None


def current_torch_device() -> torch.device:
    global _current_device
    if _current_device is None:
        _current_device = _initial_device()
        if _current_device.type == "cuda":
            torch.cuda.set_device(_current_device)
    return _current_device


def set_device(device):
    """paddle.set_device('gpu:0' | 'cpu')."""
    global _current_device
    d = _parse_device(device)
    if d.type == "cuda":
        if not _gpu_available():
            raise ValueError("no HIP/GPU device is available")
        torch.cuda.set_device(d)
        from .flags import apply_memory_limit

        apply_memory_limit(d.index or 0)  # FLAGS_gpu_memory_limit_mb / FLAGS_fraction_of_gpu_memory_to_use
    _current_device = d
    return place_of_device(d)


def get_device() -> str:
    d = current_torch_device()
    return "cpu" if d.type == "cpu" else f"gpu:{d.index or 0}"


def place_of_device(d: torch.device) -> Place:
    if d.type == "cuda":
        return CUDAPlace(d.index or 0)
    return CPUPlace()


def expected_place() -> Place:
    return place_of_device(current_torch_device())


def is_compiled_with_cuda() -> bool:
    # Paddle-ROCm builds report True here (the GPU backend is the "cuda" place).
    return _gpu_available()


def is_compiled_with_rocm() -> bool:
    return torch.version.hip is not None


def is_compiled_with_xpu() -> bool:
    return False


def is_compiled_with_custom_device(name="") -> bool:
    return False


def is_compiled_with_cinn() -> bool:
    return False


def is_compiled_with_distribute() -> bool:
    return True
