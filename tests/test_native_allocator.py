"""Native auto-growth device allocator (csrc/alloc/auto_growth.cpp) and the per-device GPUContext
(reference tests: test/cpp/fluid/memory/auto_growth_best_fit_allocator_test.cc,
stream_safe_cuda_alloc_test.cu, test/legacy_test/test_cuda_max_memory_allocated.py)."""
import os
import subprocess
import sys
import textwrap

import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd import _build


@pytest.mark.parametrize("kind", ["address", "thread"])
def test_allocator_bookkeeping_under_sanitizers(kind):
    """4 threads / 4 streams x 20k random alloc-free ops with cross-thread hand-offs: no overlap (tag check),
    no leak, allocs == frees, every chunk returned by empty_cache — under ASan+UBSan and TSan."""
    exe = _build.build_alloc_stress(kind)
    r = subprocess.run([exe, "4", "20000"], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr[-3000:]
    assert "errors=0" in r.stdout
    assert int(r.stdout.split("cross_stream_reuse=")[1].split()[0]) > 0
    assert int(r.stdout.split("deferred=")[1].split()[0]) > 0  # record_stream frees went through the deferral


def test_allocator_library_api_on_cpu():
    from paddle2_amd.device import allocator

    _build.build_allocator()
    allocator.configure(chunk_mb=64, limit_bytes=0)
    st = allocator.stats(0)
    assert set(st) >= {"allocated", "reserved", "peak_allocated", "num_chunks"}
    assert allocator.fragmentation(0)["free_blocks"] >= 0
    assert not allocator.is_active()


def test_gpu_context_pool_cpu():
    from paddle2_amd.device.context import DeviceContextPool, _device_index

    pool = DeviceContextPool.instance()
    assert pool.get(0) is pool.get("gpu:0") is paddle.device.get_context(0)
    assert _device_index(torch.device("cuda", 3)) == 3
    assert repr(pool.get(0)).startswith("GPUContext(device=0")


@pytest.mark.gpu
def test_gpu_context_streams():
    ctx = paddle.device.get_context()
    assert ctx.comm_stream() is ctx.comm_stream()
    assert ctx.h2d_stream() is not ctx.comm_stream()
    x = torch.ones(1 << 20, device="cuda")
    with torch.cuda.stream(ctx.comm_stream()):
        ctx.wait(ctx.comm_stream(), ctx.stream())
        y = x * 2
    ctx.wait(ctx.stream(), ctx.comm_stream())
    assert float(y.sum()) == 2.0 * (1 << 20)
    facts = ctx.properties()
    assert facts["num_cus"] >= 1 and facts["wavefront_size"] == 64 and "gfx" in facts["arch"]


@pytest.mark.gpu
def test_native_allocator_mem_pool_integrity():
    """A torch MemPool backed by the native allocator inside a caching-allocator process (FLAGS=0): random
    sized live tensors keep their contents and the native chunk pool grows."""
    script = textwrap.dedent("""
        import torch
        from paddle2_amd.device import allocator
        allocator.configure(chunk_mb=64, limit_bytes=0)
        before = allocator.stats(torch.cuda.current_device())
        pool = allocator.mem_pool()
        g = torch.Generator().manual_seed(0)
        live = []
        with torch.cuda.use_mem_pool(pool):
            for i in range(200):
                n = int(torch.randint(1, 1 << 22, (1,), generator=g))
                t = torch.full((n,), float(i % 97), device="cuda")
                live.append((i, t))
                if i % 3 == 0:
                    live.pop(int(torch.randint(0, len(live), (1,), generator=g)))
            torch.cuda.synchronize()
            for i, t in live:
                assert float(t.min()) == float(i % 97) == float(t.max())
        after = allocator.stats(torch.cuda.current_device())
        assert after["num_grow"] > before["num_grow"] and after["reserved"] > 0
        del live, t, pool          # release the pool's segments while the HIP runtime is alive
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        print("OK")
    """)
    env = dict(os.environ, FLAGS_use_native_allocator="0")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0 and "OK" in r.stdout, r.stderr[-3000:]


@pytest.mark.gpu
def test_native_allocator_is_default_and_supports_graph_capture():
    """The native allocator is the process default on the GPU (FLAGS unset), and hipGraph capture gets a
    private pool from it: a captured step replays correctly after other allocations reuse freed memory."""
    script = textwrap.dedent("""
        import json, torch
        import paddle2_amd as paddle
        from paddle2_amd.device import allocator
        x = torch.randn(1024, 1024, device="cuda")
        w = torch.randn(1024, 1024, device="cuda")
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                y = torch.relu(x @ w) + 1.0
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            y = torch.relu(x @ w) + 1.0
            z = y * 2.0
        junk = [torch.randn(512, 512, device="cuda") for _ in range(20)]   # reuse of freed general memory
        del junk
        x.copy_(torch.randn(1024, 1024, device="cuda"))
        g.replay()
        torch.cuda.synchronize()
        ref = (torch.relu(x @ w) + 1.0) * 2.0
        ok = bool(torch.allclose(z, ref, atol=1e-3, rtol=1e-3))
        del g
        torch.cuda.synchronize()
        print(json.dumps({"active": allocator.is_active(), "hooked": allocator.has_record_stream(), "ok": ok,
                          "peak": paddle.device.cuda.max_memory_allocated()}))
    """)
    env = dict(os.environ)
    env.pop("FLAGS_use_native_allocator", None)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["active"] and res["hooked"] and res["ok"] and res["peak"] > 0, res


@pytest.mark.gpu
def test_native_allocator_process_wide_training():
    """FLAGS_use_native_allocator=1: a fresh process trains an MLP with a side-stream copy on the native
    allocator; the loss trajectory equals the caching allocator's and the stats API reports its usage."""
    script = textwrap.dedent("""
        import json, os, sys
        import numpy as np
        import torch
        import paddle2_amd as paddle
        from paddle2_amd.device import allocator
        paddle.seed(0)
        net = paddle.nn.Sequential(paddle.nn.Linear(256, 512), paddle.nn.ReLU(), paddle.nn.Linear(512, 10))
        opt = paddle.optimizer.AdamW(1e-3, parameters=net.parameters())
        rs = np.random.RandomState(0)
        losses = []
        ctx = paddle.device.get_context()
        for step in range(20):
            xh = torch.from_numpy(rs.randn(64, 256).astype("float32")).pin_memory()
            with torch.cuda.stream(ctx.h2d_stream()):
                xd = xh.to("cuda", non_blocking=True)
            torch.cuda.current_stream().wait_stream(ctx.h2d_stream())
            xd.record_stream(torch.cuda.current_stream())
            x = paddle.Tensor._wrap(xd)
            y = paddle.to_tensor(rs.randint(0, 10, (64,)).astype("int64")).cuda()
            loss = paddle.nn.functional.cross_entropy(net(x), y)
            loss.backward(); opt.step(); opt.clear_grad()
            losses.append(float(loss))
        torch.cuda.synchronize()
        st = allocator.stats(0) if allocator.is_active() else {}
        print(json.dumps({"active": allocator.is_active(), "losses": losses, "stats": st,
                          "api_alloc": paddle.device.cuda.memory_allocated(),
                          "api_peak": paddle.device.cuda.max_memory_allocated()}))
    """)
    import json

    res = {}
    for mode in ("native", "caching"):
        env = dict(os.environ)
        env["FLAGS_use_native_allocator"] = "1" if mode == "native" else "0"
        r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
        assert r.returncode == 0, r.stderr[-3000:]
        res[mode] = json.loads(r.stdout.strip().splitlines()[-1])
    nat, cach = res["native"], res["caching"]
    assert nat["active"] and not cach["active"]
    assert nat["losses"] == pytest.approx(cach["losses"], rel=1e-5, abs=1e-6)
    st = nat["stats"]
    assert st["num_allocs"] > 100 and st["reserved"] >= st["peak_allocated"] > 0
    assert nat["api_peak"] == st["peak_allocated"] and nat["api_alloc"] == st["allocated"]


@pytest.mark.gpu
def test_native_allocator_record_stream_fences_side_stream_reader():
    """Tensor.record_stream reaches the native allocator (C++ install): a tensor freed on the main stream while a
    slow side stream still reads it must not be handed to the next main-stream allocation before that read."""
    script = textwrap.dedent("""
        import json
        import torch
        import paddle2_amd as paddle
        from paddle2_amd.device import allocator
        assert allocator.is_active() and allocator.has_record_stream()
        main = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        bad = 0
        for it in range(20):
            a = torch.full((1 << 20,), float(it + 1), device="cuda")
            out = torch.empty_like(a)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                torch.cuda._sleep(20_000_000)    # the side stream reads `a` only after ~10 ms
                out.copy_(a)
            a.record_stream(side)
            del a                                # freed on the main stream while the side read is pending
            b = torch.full((1 << 20,), -7.0, device="cuda")   # would reuse a's block without the fence
            torch.cuda.synchronize()
            bad += int((out != float(it + 1)).sum())
            del b, out
        st = allocator.stats(0)
        print(json.dumps({"bad": bad, "record_stream": st["record_stream"], "deferred": st["deferred_frees"]}))
    """)
    import json

    env = dict(os.environ, FLAGS_use_native_allocator="1")
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["bad"] == 0 and res["record_stream"] >= 20 and res["deferred"] >= 20, res


@pytest.mark.gpu
def test_native_allocator_torch_stats_and_miopen_workspace():
    """torch.cuda memory stats answer from the native allocator, and MIOpen convolutions get a workspace bound
    from its cacheInfo (a throwing cacheInfo bounded the workspace at 0 and MIOpen fell back to its naive direct
    kernels, ~100x slower): a ResNet-sized bf16 NHWC 3x3 conv must run at GEMM speed."""
    script = textwrap.dedent("""
        import json, time, torch
        import paddle2_amd  # noqa: F401  (installs the native allocator)
        from paddle2_amd.device import allocator
        torch.cuda.reset_peak_memory_stats()
        x = torch.randn(256, 64, 56, 56, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        w = torch.randn(64, 64, 3, 3, device="cuda", dtype=torch.bfloat16).to(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w.requires_grad_(True)
        for _ in range(3):
            y = torch.nn.functional.conv2d(x, w, padding=1)
            y.backward(torch.ones_like(y))
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(5):
            y = torch.nn.functional.conv2d(x, w, padding=1)
            y.backward(torch.ones_like(y))
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t) / 5 * 1e3
        st = torch.cuda.memory_stats()
        print(json.dumps({"active": allocator.is_active(), "ms": ms, "peak": torch.cuda.max_memory_allocated(),
                          "reserved": torch.cuda.memory_reserved(), "cur": st.get("allocated_bytes.all.current", 0)}))
    """)
    env = dict(os.environ)
    env.pop("FLAGS_use_native_allocator", None)
    r = subprocess.run([sys.executable, "-c", script], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr[-3000:]
    import json

    res = json.loads(r.stdout.strip().splitlines()[-1])
    # fwd + dgrad + wgrad = 3 x 2*256*56*56*64*64*9 = 44 GFLOP: 30 ms is < 1.5 TF/s (naive kernels take seconds)
    assert res["active"] and res["peak"] > 0 and res["reserved"] >= res["cur"] > 0, res
    assert res["ms"] < 30.0, res


@pytest.mark.gpu
def test_native_allocator_oom_raises_torch_error():
    """An allocation the device cannot hold raises torch.OutOfMemoryError (through the torch hook), never hands torch
    a null pointer — a null data pointer for a non-empty tensor turned a 7B out-of-memory into a GPU memory-access
    fault.  torch.empty launches no kernel, so the check itself cannot touch the device."""
    import torch

    from paddle2_amd.device import allocator

    if not allocator.is_active():
        pytest.skip("native allocator not active")
    total = torch.cuda.get_device_properties(0).total_memory
    before = allocator.stats(0)["num_oom_retries"]
    with pytest.raises(torch.OutOfMemoryError):
        torch.empty(int(total * 1.5) // 2, dtype=torch.bfloat16, device="cuda")
    assert allocator.stats(0)["num_oom_retries"] == before + 1
    x = torch.ones(1024, device="cuda")   # the allocator still serves after the failure
    assert float(x.sum()) == 1024.0
