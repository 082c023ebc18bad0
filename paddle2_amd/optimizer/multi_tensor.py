"""Device-resident multi-tensor tables for the fused optimizer / AMP / clip kernels.

The table (one 56-byte record per tensor: param, grad, moment1, moment2, master, numel,
lr_ratio, decay) and its chunk prefix are uploaded once per parameter set; every step then is
a single persistent-kernel launch per dtype group (csrc/kernels/optim.hip).
"""
from __future__ import annotations

import numpy as np
import torch

from ..ops import _native as N

_META = np.dtype([("p", "<u8"), ("g", "<u8"), ("m", "<u8"), ("v", "<u8"), ("master", "<u8"), ("n", "<i8"),
                  ("lr_ratio", "<f4"), ("decay", "<f4")])
assert _META.itemsize == 56


class MultiTensorTable:
    def __init__(self, params, grads, m=None, v=None, master=None, lr_ratio=None, decay=None):
        C = N.require()
        assert C.opt_meta_bytes() == _META.itemsize
        self.C = C
        self.chunk = C.opt_chunk_size()
        T = len(params)
        rec = np.zeros(T, dtype=_META)
        prefix = np.zeros(T + 1, dtype=np.int64)
        for i in range(T):
            rec[i]["p"] = params[i].data_ptr() if params[i] is not None else 0
            rec[i]["g"] = grads[i].data_ptr()
            rec[i]["m"] = m[i].data_ptr() if m is not None else 0
            rec[i]["v"] = v[i].data_ptr() if v is not None else 0
            rec[i]["master"] = master[i].data_ptr() if (master is not None and master[i] is not None) else 0
            n = grads[i].numel()
            rec[i]["n"] = n
            rec[i]["lr_ratio"] = 1.0 if lr_ratio is None else lr_ratio[i]
            rec[i]["decay"] = 0.0 if decay is None else decay[i]
            prefix[i + 1] = prefix[i] + (n + self.chunk - 1) // self.chunk
        dev = grads[0].device
        self.T = T
        self.chunks = int(prefix[-1])
        self.meta = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
        self.prefix = torch.from_numpy(prefix).to(dev)
        self.gdt = N.DT_CODE[grads[0].dtype]
        self.pdt = N.DT_CODE[params[0].dtype] if params[0] is not None else self.gdt
        self.device = dev
        self.has_master = master is not None and any(x is not None for x in master)
        # Keep the persistent storages (params, moments, master weights) alive for the table's
        # lifetime.  Gradients are NOT referenced: they are re-created every step (lazy-zero
        # clear_grad) and callers re-validate a cached table against the current grad pointers, so
        # holding them here would pin a whole extra gradient set in HBM.
        self._refs = (params, m, v, master)

    @classmethod
    def for_grads(cls, grads):
        return cls([None] * len(grads), grads)

    def adamw(self, lr, beta1, beta2, eps, bc1, bc2, found_inf=None, inv_scale=None):
        self.C.adamw_mt(self.pdt, self.gdt, int(self.has_master), self.meta.data_ptr(), self.prefix.data_ptr(), self.T,
                        self.chunks, float(lr), float(beta1), float(beta2), float(eps), float(bc1), float(bc2),
                        N.ptr(found_inf), N.ptr(inv_scale), N.stream())

    def sqnorm(self):
        out = torch.zeros(1, dtype=torch.float32, device=self.device)
        self.C.sqnorm_mt(self.gdt, self.meta.data_ptr(), self.prefix.data_ptr(), self.T, self.chunks, out.data_ptr(),
                         N.stream())
        return out

    def scale(self, coef):
        self.C.scale_mt(self.gdt, self.meta.data_ptr(), self.prefix.data_ptr(), self.T, self.chunks, coef.data_ptr(),
                        N.stream())

    def unscale(self, scale, found_inf):
        self.C.unscale_mt(self.gdt, self.meta.data_ptr(), self.prefix.data_ptr(), self.T, self.chunks,
                          scale.data_ptr(), found_inf.data_ptr(), N.stream())


def aligned16(t) -> bool:
    return t is None or t.data_ptr() % 16 == 0
