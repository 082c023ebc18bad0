import torch, sys
sys.path.insert(0,'.')
from paddle2_amd.ops import torch_ops as T
from paddle2_amd.ops import _native as N
def t(fn, it=20):
    for _ in range(3): fn()
    torch.cuda.synchronize(); s=torch.cuda.Event(enable_timing=True); e=torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it): fn()
    e.record(); torch.cuda.synchronize(); return s.elapsed_time(e)/it
M,H=32768,11008
gu=torch.randn(M,2*H,device='cuda',dtype=torch.bfloat16); da=torch.randn(M,H,device='cuda',dtype=torch.bfloat16)
dgu=torch.empty_like(gu); dT=torch.empty(2*H,M,device='cuda',dtype=torch.bfloat16)
C=N.native()
f1=lambda: C.swiglu_bwd_t(gu.data_ptr(),da.data_ptr(),dgu.data_ptr(),dT.data_ptr(),M,H,2*H,N.stream())
def f2():
    C.swiglu_bwd(1, gu.data_ptr(), gu.data_ptr()+H*2, da.data_ptr(), dgu.data_ptr(), dgu.data_ptr()+H*2, M, H, 2*H, 2*H, 2*H, 2*H, N.stream())
    T.transpose2d(dgu)
f3=lambda: C.swiglu_bwd(1, gu.data_ptr(), gu.data_ptr()+H*2, da.data_ptr(), dgu.data_ptr(), dgu.data_ptr()+H*2, M, H, 2*H, 2*H, 2*H, 2*H, N.stream())
print("bwd_t", t(f1), "bwd+transpose", t(f2), "bwd", t(f3))
