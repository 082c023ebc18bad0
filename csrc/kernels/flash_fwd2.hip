// The two-row-block flash forward (fwd_kernel<128, *, *, false, *, 4, 2>, see flash_attn.hip): its own translation
// unit so it can be built with the VGPR form of the MFMA instructions (-mllvm -amdgpu-mfma-vgpr-form, set for this
// file by paddle2_amd/_build.py).  The kernel pins its O accumulators to AGPRs itself; without the flag hipcc also
// homes the score accumulators in AGPRs and copies 64 of them to VGPRs for the softmax on every key tile.
#define PD_FA_DEVICE_ONLY
#include "flash_attn.hip"

namespace pd {
namespace fa {

void launch_fwd_rb2(bool f16, bool causal, int mode, dim3 grid, hipStream_t st, const void* q, const void* k,
                    const void* v, void* o, float* lse, int B, int Sq, int Sk, int Hq, int Hk, long sq, long sk, long sv,
                    long so, float scale, const Ext& ex) {
#define PD_FA_RB2(FF, CC, MM)                                                                                       \
  fwd_kernel<128, CC, MM, false, FF, 4, 2><<<grid, 256, 0, st>>>((const bf16*)q, (const bf16*)k, (const bf16*)v,  \
                                                                 (bf16*)o, lse, B, Sq, Sk, Hq, Hk, sq, sk, sv, so,   \
                                                                 scale, ex)
#define PD_FA_RB2_M(FF, CC) \
  if (mode == 0) PD_FA_RB2(FF, CC, kDense); else PD_FA_RB2(FF, CC, kVarlen);
  if (f16) { if (causal) { PD_FA_RB2_M(true, true) } else { PD_FA_RB2_M(true, false) } }
  else { if (causal) { PD_FA_RB2_M(false, true) } else { PD_FA_RB2_M(false, false) } }
#undef PD_FA_RB2_M
#undef PD_FA_RB2
}

}  // namespace fa
}  // namespace pd
