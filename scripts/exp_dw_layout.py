import torch, json
def t(fn, it=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize()
    return s.elapsed_time(e) / it
M=32768
for name,(K,N) in {"qkv": (4096, 12288), "o": (4096, 4096), "gate_up": (4096, 22016), "down": (11008, 4096), "lm_head": (4096, 32000)}.items():
    x = torch.randn(M, K, device="cuda", dtype=torch.bfloat16)
    dy = torch.randn(M, N, device="cuda", dtype=torch.bfloat16)
    base = t(lambda: x.t() @ dy)
    tx = t(lambda: x.t().contiguous())
    tdy = t(lambda: dy.t().contiguous())
    xT = x.t().contiguous(); dyT = dy.t().contiguous()
    fast = t(lambda: xT @ dyT.t())
    alt = t(lambda: (dy.t() @ x))  # dW^T directly
    print(json.dumps(dict(name=name, base=round(base,3), tx=round(tx,3), tdy=round(tdy,3), fast=round(fast,3), total=round(tx+tdy+fast,3), dWT=round(alt,3))), flush=True)
