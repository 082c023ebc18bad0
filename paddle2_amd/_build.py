"""Build the native extensions: ``paddle2_amd._C`` (HIP kernels for gfx950 + pybind11 host glue) and
``paddle2_amd._runtime`` (host-only C++ runtime: TCPStore, comm watchdog, host tracer, blocking queue).

Invoked by ``__graft_entry__.build()`` and ``python -m paddle2_amd._build``.  Objects are cached
by content hash under ``build/`` so a rebuild only recompiles what changed.  Everything targets
``--offload-arch=gfx950`` (MI355X / CDNA4) only.
"""
from __future__ import annotations

import hashlib
import os
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "csrc")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("PADDLE2_AMD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path():
    return os.path.join(ROOT, "paddle2_amd", "_C" + _ext_suffix())


def _sources():
    kdir = os.path.join(CSRC, "kernels")
    hips = sorted(os.path.join(kdir, f) for f in os.listdir(kdir) if f.endswith(".hip"))
    return hips, os.path.join(CSRC, "bindings.cpp")


# per-translation-unit extras: flash_fwd2.hip includes flash_attn.hip and needs the VGPR form of the MFMAs
_TU_FLAGS = {"flash_fwd2.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form=1"]}
_TU_DEPS = {"flash_fwd2.hip": ["flash_attn.hip"]}


def _hash(path, extra=""):
    h = hashlib.sha1()
    with open(path, "rb") as f:
        h.update(f.read())
    for dep in _TU_DEPS.get(os.path.basename(path), []):
        with open(os.path.join(os.path.dirname(path), dep), "rb") as f:
            h.update(f.read())
    # headers affect every translation unit
    kdir = os.path.join(CSRC, "kernels")
    for hf in sorted(os.listdir(kdir)):
        if hf.endswith(".h"):
            with open(os.path.join(kdir, hf), "rb") as f:
                h.update(f.read())
    h.update(extra.encode())
    return h.hexdigest()[:16]


def _run(cmd):
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return r


def build(verbose=False, jobs=None):
    os.makedirs(BUILD, exist_ok=True)
    hips, binding = _sources()
    hip_flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-munsafe-fp-atomics",
                 "-I", os.path.join(CSRC, "kernels")]
    import pybind11

    py_inc = sysconfig.get_paths()["include"]
    host_flags = ["-O2", "-std=c++17", "-fPIC", "-I", py_inc, "-I", pybind11.get_include()]

    def compile_one(src):
        is_hip = src.endswith(".hip")
        flags = (hip_flags + _TU_FLAGS.get(os.path.basename(src), [])) if is_hip else host_flags
        key = _hash(src, " ".join(flags))
        obj = os.path.join(BUILD, os.path.basename(src) + "." + key + ".o")
        if not os.path.exists(obj):
            if is_hip:
                cmd = [HIPCC] + flags + ["-c", src, "-o", obj]
            else:
                cmd = ["g++"] + flags + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            _run(cmd)
        return obj

    srcs = hips + [binding]
    with ThreadPoolExecutor(max_workers=jobs or min(8, len(srcs))) as ex:
        objs = list(ex.map(compile_one, srcs))
    out = target_path()
    link_key = hashlib.sha1("".join(objs).encode()).hexdigest()[:16]
    stamp = out + ".stamp"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == link_key:
        return out
    tmp = out + ".tmp"
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}"] + objs + ["-o", tmp]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(link_key)
    return out


def runtime_target_path():
    return os.path.join(ROOT, "paddle2_amd", "_runtime" + _ext_suffix())


def build_runtime(verbose=False):
    """Host-only runtime module (g++, pybind11, pthreads); no HIP so it loads on CPU machines too."""
    rdir = os.path.join(CSRC, "runtime")
    srcs = sorted(os.path.join(rdir, f) for f in os.listdir(rdir) if f.endswith(".cpp"))
    import pybind11

    flags = ["-O2", "-std=c++17", "-fPIC", "-I", sysconfig.get_paths()["include"], "-I", pybind11.get_include(),
             "-I", rdir]
    h = hashlib.sha1(" ".join(flags).encode())
    for f in sorted(os.listdir(rdir)):
        if os.path.isfile(os.path.join(rdir, f)):
            with open(os.path.join(rdir, f), "rb") as fh:
                h.update(fh.read())
    key = h.hexdigest()[:16]
    out = runtime_target_path()
    stamp = out + ".stamp"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    os.makedirs(BUILD, exist_ok=True)

    def comp(src):
        obj = os.path.join(BUILD, "rt_" + os.path.basename(src) + "." + key + ".o")
        if not os.path.exists(obj):
            cmd = ["g++"] + flags + ["-c", src, "-o", obj]
            if verbose:
                print(" ".join(cmd), flush=True)
            _run(cmd)
        return obj

    with ThreadPoolExecutor(max_workers=min(8, len(srcs))) as ex:
        objs = list(ex.map(comp, srcs))
    tmp = out + ".tmp"
    _run(["g++", "-shared", "-fPIC"] + objs + ["-o", tmp, "-lpthread"])
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return out


def rccl_target_path():
    return os.path.join(ROOT, "paddle2_amd", "_rccl" + _ext_suffix())


def build_rccl(verbose=False):
    """ProcessGroupRCCL core (csrc/comm/rccl_group.cpp): host C++ against the HIP runtime and librccl, pybind11."""
    import pybind11

    src = os.path.join(CSRC, "comm", "rccl_group.cpp")
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include",
             "-I", sysconfig.get_paths()["include"], "-I", pybind11.get_include()]
    libs = ["-L/opt/rocm/lib", "-lrccl", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    key = _hash(src, " ".join(flags + libs) + open(os.path.join(CSRC, "comm", "rccl_core.h")).read())
    out = rccl_target_path()
    stamp = out + ".stamp"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    tmp = out + ".tmp"
    cmd = ["g++"] + flags + [src, "-o", tmp] + libs
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return out


def alloc_target_path():
    return os.path.join(ROOT, "paddle2_amd", "_pd_alloc.so")


def build_allocator(verbose=False):
    """Native auto-growth device allocator (csrc/alloc/auto_growth.cpp): a plain C-ABI shared library loaded by
    torch's CUDAPluggableAllocator and by ctypes (stats).  Host code against the HIP runtime."""
    src = os.path.join(CSRC, "alloc", "auto_growth.cpp")
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include"]
    key = _hash(src, " ".join(flags))
    out = alloc_target_path()
    stamp = out + ".stamp"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    tmp = out + ".tmp"
    cmd = ["g++"] + flags + [src, "-o", tmp, "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath,/opt/rocm/lib"]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return out


def alloc_torch_target_path():
    return os.path.join(ROOT, "paddle2_amd", "_pd_alloc_torch.so")


def build_alloc_torch(verbose=False):
    """The torch-side installer of the native allocator (csrc/alloc/torch_hook.cpp): builds torch's pluggable
    allocator in C++ with the record-stream hook wired to pd_alloc_record_stream.  Links libtorch_hip and resolves
    the pd_alloc_* symbols from _pd_alloc.so (loaded RTLD_GLOBAL first)."""
    import torch

    src = os.path.join(CSRC, "alloc", "torch_hook.cpp")
    tdir = os.path.dirname(torch.__file__)
    abi = int(torch._C._GLIBCXX_USE_CXX11_ABI)
    flags = ["-O2", "-std=c++17", "-fPIC", "-shared", "-D__HIP_PLATFORM_AMD__", "-DUSE_ROCM",
             f"-D_GLIBCXX_USE_CXX11_ABI={abi}", "-I", "/opt/rocm/include", "-I", os.path.join(tdir, "include"),
             "-I", os.path.join(tdir, "include", "torch", "csrc", "api", "include")]
    key = _hash(src, " ".join(flags))
    out = alloc_torch_target_path()
    stamp = out + ".stamp"
    if os.path.exists(out) and os.path.exists(stamp) and open(stamp).read() == key:
        return out
    tmp = out + ".tmp"
    lib = os.path.join(tdir, "lib")
    cmd = ["g++"] + flags + [src, "-o", tmp, "-L" + lib, "-ltorch_hip", "-lc10_hip", "-lc10", "-ltorch_cpu",
                             "-L/opt/rocm/lib", "-lamdhip64", "-Wl,-rpath," + lib, "-Wl,-rpath,/opt/rocm/lib",
                             "-Wl,--allow-shlib-undefined"]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(key)
    return out


def build_alloc_stress(kind="address", verbose=False):
    """The allocator's bookkeeping + the multi-threaded stress driver, against the fake HIP header (host memory,
    asynchronous events), under ``kind`` = "address" (ASan+UBSan) or "thread" (TSan).  CPU-only."""
    adir = os.path.join(CSRC, "alloc")
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, f"alloc_stress_{kind}")
    cmd = (["g++", "-O1", "-g", "-std=c++17", "-I", os.path.join(adir, "test", "fake_hip")] + _SAN_FLAGS[kind]
           + [os.path.join(adir, "auto_growth.cpp"), os.path.join(adir, "test", "alloc_stress.cpp"), "-o", out,
              "-lpthread"])
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    return out


_SAN_FLAGS = {
    "thread": ["-fsanitize=thread"],
    "address": ["-fsanitize=address,undefined", "-fno-omit-frame-pointer", "-fno-sanitize-recover=undefined"],
}


def build_sanitized(kind="thread", verbose=False):
    """Sanitizer build of the host runtime (store, watchdog, tracer) linked into the stress driver
    csrc/runtime/stress/runtime_stress.cpp: ``kind`` "thread" (TSan, data races) or "address" (ASan + UBSan).
    Host code only — GPU sanitizers are not used on this hardware.  Returns the executable path."""
    rdir = os.path.join(CSRC, "runtime")
    srcs = [os.path.join(rdir, f) for f in ("tcp_store.cpp", "watchdog.cpp", "tracer.cpp", "fleet_executor.cpp")]
    srcs.append(os.path.join(rdir, "stress", "runtime_stress.cpp"))
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, f"runtime_stress_{kind}")
    cmd = ["g++", "-O1", "-g", "-std=c++17", "-I", rdir] + _SAN_FLAGS[kind] + srcs + ["-o", out, "-lpthread", "-ldl"]
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    return out


def build_rccl_stress(kind="thread", verbose=False):
    """The ProcessGroupRCCL core (csrc/comm/rccl_core.h) + its 4-rank stress driver (csrc/comm/test/rccl_stress.cpp)
    against the threaded fake RCCL / HIP (csrc/comm/test/fake/), under ``kind`` = "thread" (TSan) or "address"
    (ASan + UBSan).  CPU-only; returns the executable path."""
    cdir = os.path.join(CSRC, "comm")
    os.makedirs(BUILD, exist_ok=True)
    out = os.path.join(BUILD, f"rccl_stress_{kind}")
    cmd = (["g++", "-O1", "-g", "-std=c++17", "-I", os.path.join(cdir, "test", "fake")] + _SAN_FLAGS[kind]
           + [os.path.join(cdir, "test", "rccl_stress.cpp"), "-o", out, "-lpthread"])
    if verbose:
        print(" ".join(cmd), flush=True)
    _run(cmd)
    return out


def build_all(verbose=False):
    alloc = build_allocator(verbose=verbose)
    build_alloc_torch(verbose=verbose)
    build_rccl(verbose=verbose)
    return build(verbose=verbose), build_runtime(verbose=verbose), alloc


if __name__ == "__main__":
    print(build_all(verbose="-v" in sys.argv))
