"""SwiGLU forward / backward at the Llama-2-7B MLP shape (32768 rows, H 11008, packed gate|up) with 2 or 4 rows per
kernel iteration (PADDLE2_AMD_SWIGLU_ROWS, read per launch): ms, TB/s and bitwise equality of the two forms."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from paddle2_amd.ops import _native as N  # noqa: E402


def timeit(fn, iters=10):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        best = min(best, s.elapsed_time(e) / iters)
    return best


def main():
    M, H = 32768, 11008
    g = torch.Generator(device="cuda").manual_seed(0)
    gu = torch.randn(M, 2 * H, device="cuda", generator=g).to(torch.bfloat16)
    dout = torch.randn(M, H, device="cuda", generator=g).to(torch.bfloat16)
    C = N.native()
    bf = 1   # kBF16
    outs = {}
    for rnd in range(2):
        for rows in ("2", "4"):
            os.environ["PADDLE2_AMD_SWIGLU_ROWS"] = rows
            out = torch.empty(M, H, device="cuda", dtype=torch.bfloat16)
            dgu = torch.empty_like(gu)
            fwd = lambda: C.swiglu_fwd(bf, gu.data_ptr(), gu.data_ptr() + 2 * H, out.data_ptr(), M, H, 2 * H, 2 * H,  # noqa: E731
                                       N.stream())
            bwd = lambda: C.swiglu_bwd(bf, gu.data_ptr(), gu.data_ptr() + 2 * H, dout.data_ptr(), dgu.data_ptr(),  # noqa: E731
                                       dgu.data_ptr() + 2 * H, M, H, 2 * H, 2 * H, 2 * H, 2 * H, N.stream())
            tf, tb = timeit(fwd), timeit(bwd)
            fwd(); bwd()
            torch.cuda.synchronize()
            outs[rows] = (out.clone(), dgu.clone())
            eq = all(torch.equal(a, b) for a, b in zip(outs[rows], outs["2"]))
            print(json.dumps({"rows": int(rows), "round": rnd, "fwd_ms": round(tf, 4), "fwd_TBs": round(3 * M * H * 2 / tf / 1e9, 2),
                              "bwd_ms": round(tb, 4), "bwd_TBs": round(5 * M * H * 2 / tb / 1e9, 2),
                              "equal_to_rows2": eq}), flush=True)
    os.environ.pop("PADDLE2_AMD_SWIGLU_ROWS", None)


if __name__ == "__main__":
    main()
