"""paddle.version."""
full_version = "3.0.0"
major, minor, patch = "3", "0", "0"
rc = "0"
istaged = True
commit = "mi355x-native"
with_mkl = "OFF"
cuda_version = "False"
cudnn_version = "False"
import torch as _t
hip_version = str(_t.version.hip)
xpu_version = "False"


def show():
    print(f"full_version: {full_version}\nhip: {hip_version}\ncommit: {commit}")


def cuda():
    return cuda_version


def cudnn():
    return cudnn_version
