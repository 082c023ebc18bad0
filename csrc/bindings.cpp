// pybind11 module `paddle2_amd._C`: thin host entry points for the CDNA4 kernels.
//
// Tensors cross the boundary as raw device pointers (ints) + shapes + the caller's HIP stream
// handle, so this module does not depend on libtorch's C++ ABI (it is built with hipcc alone
// and loads into the process after torch has brought up the HIP runtime). Every entry point is
// asynchronous on the given stream and safe to capture in a hipGraph (no allocation, no sync).
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <tuple>
#include <vector>

#include <cstdint>
#include <stdexcept>
#include <string>

namespace py = pybind11;

extern "C" {
int pd_norm_fwd(int, int, int, const void*, const void*, const void*, const void*, void*, void*, float*, float*, int,
                int, float, void*);
int pd_norm_bwd_blocks(int);
int pd_bias_grad_chunks(int, int);
int pd_bias_grad(int, int, const void*, float*, void*, int, int, int, void*);
int pd_norm_bwd(int, int, int, const void*, const void*, const void*, const float*, const float*, const void*, void*,
                float*, float*, void*, void*, int, int, int, int, int, int, void*);
int pd_swiglu_fwd(int, const void*, const void*, void*, long, int, long, long, void*);
int pd_gemm(int, int, const void*, long, const void*, long, void*, long, void*, long, const void*, int, int, int, float,
            int, int, int, void*, long, void*);
int pd_gemm_grouped(int, int, const void*, long, const void*, long, long, void*, long, long, void*, long, const void*,
                    long, const int*, int, int, int, int, int, int, float, int, int, void*);
int pd_transpose16(const void*, void*, long, long, long, long, void*);
int pd_gemm_conv(const void*, long, const void*, const void*, const void*, long, void*, long, int, int, int, int,
                 int, int, int, int, int, int, int, int, void*);
void pd_gemm_set_rope(const float*, const float*, int, int);
int pd_gemm_f8(int, int, int, const void*, long, const void*, long, void*, long, const void*, const float*,
               const float*, int, int, int, float, int, int, void*, long, void*);
long pd_ar_sig_bytes();
int pd_bias_act(int, int, int, const void*, const void*, void*, long, int, long, long, void*);
int pd_bias_act_bwd(int, int, int, const void*, const void*, const void*, void*, long, int, long, long, void*);
int pd_dropout_add(int, int, const void*, const void*, void*, long, unsigned, float, void*);
int pd_memcpy_d2d(void*, const void*, long, void*);
int pd_ar_alloc(long, void**);
int pd_ar_free(void*);
int pd_ar_get_handle(void*, void*);
int pd_ar_open_handle(const void*, void**);
int pd_ar_close_handle(void*);
int pd_ar_allreduce(int, int, const void* const*, const void* const*, int, int, void*, long, long, long, unsigned,
                    unsigned*, int, int, void*);
int pd_swiglu_bwd_t(const void*, const void*, void*, void*, long, int, long, void*);
int pd_swiglu_bwd(int, const void*, const void*, const void*, void*, void*, long, int, long, long, long, long, void*);
int pd_rope(int, int, int, const void*, void*, const float*, const float*, const int64_t*, int, int, int, int, int,
            long, long, void*);
int pd_opt_chunk_size();
int pd_opt_meta_bytes();
int pd_adamw_mt(int, int, int, const void*, const long*, int, long, float, float, float, float, float, float,
                const float*, const float*, void*);
int pd_unscale_mt(int, const void*, const long*, int, long, const float*, float*, void*);
int pd_sqnorm_mt(int, const void*, const long*, int, long, float*, void*);
int pd_scale_mt(int, const void*, const long*, int, long, const float*, void*);
int pd_update_loss_scaling(const float*, float*, int*, int*, int, int, float, float, void*);
int pd_softmax_mask_fwd(int, int, const void*, const void*, void*, long, int, int, int, void*);
int pd_softmax_mask_bwd(int, const void*, const void*, void*, long, int, void*);
int pd_ce_stats(int, const void*, const int64_t*, float*, float*, float*, long, long, long, void*);
int pd_ce_bwd(int, const void*, const int64_t*, const float*, const float*, void*, long, long, long, long, int, void*);
int pd_embed_fwd(int, const int64_t*, const void*, void*, long, int, long, long, void*);
int pd_embed_bwd(int, const int64_t*, const void*, float*, long, int, long, long, long, void*);
int pd_cast_from_f32(int, const float*, void*, long, void*);
int pd_fp8_cast(int, int, const void*, void*, void*, long, long, const float*, float*, float*, void*);
int pd_colsum(int, const float*, void*, int, int, int, void*);
int pd_fp8_update_scale(int, float* const*, const int*, float* const*, float* const*, float* const*, float* const*,
                        const float*, const float*, void*);
int pd_decode_attn(const void*, long, long, const void*, const void*, long, long, long, const int*, int, int,
                   const int*, int, float*, float*, void*, long, long, int, int, int, int, int, float, int, void*);
int pd_cache_write(const void*, const void*, long, long, void*, void*, long, long, long, const int*, int, int,
                   const int*, const int*, int, int, int, void*);
long pd_bn_workspace(int, long, int);
int pd_wo_splits(int, int, int, int);
int pd_dec_splits(int, int, int);
int pd_dec_gemm(const void*, const void*, const void*, void*, float*, int, int, int, int, int, int*, void*, int);
int pd_dec_reduce(const float*, int, int, int, const void*, void*, void*);
int pd_norm_fwd_part(int, const float*, int, const void*, const void*, void*, void*, int, int, float, void*);
int pd_dec64_gemm(const void*, const void*, const void*, void*, int, int, int, int, int, void*);
int pd_dec64_rt(int);
int pd_dec64s_gemm(const void*, const void*, const void*, void*, float*, int, int, int, int, int, int, void*);
long pd_dec64s_workspace(int, int, int, int, int, int);
long pd_wo_workspace(int, int, int);
int pd_wo_gemm(int, const void*, const void*, const float*, const float*, int, const void*, void*, float*, int, int, int,
               int, void*);
int pd_bn_fwd_train(int, const void*, const void*, void*, long, int, float*, float*, const float*, const float*, float,
                    float, float*, float*, float*, int, int, void*);
int pd_bn_apply(int, const void*, const void*, void*, long, int, const float*, const float*, int, void*);
int pd_bn_bwd(int, const void*, const void*, const void*, const float*, const float*, const float*, void*, void*,
              float*, float*, long, int, float*, int, void*);
int pd_flash_fwd_ext(int, const void*, const void*, const void*, void*, float*, int, int, int, int, int, int, long,
                     long, long, long, float, int, int, const int*, const int*, int, const int*, const int*, const int*,
                     int, int, unsigned, float, void*);
int pd_flash_bwd_ext(int, const void*, const void*, const void*, const void*, const void*, const float*, float*, void*,
                     void*, void*, float*, int, int, int, int, int, int, long, long, long, long, long, long, long, float,
                     int, int, const int*, const int*, int, const int*, const int*, const int*, int, int, unsigned,
                     float, void*);
int pd_flash_fwd(int, const void*, const void*, const void*, void*, float*, int, int, int, int, int, int, long, long,
                 long, long, float, int, void*);
int pd_flash_bwd_block(int);
void pd_flash_bwd_set_rope(const float*, const float*);
long pd_flash_ds_elems(int, int, int, int, int, int);
void pd_flash_bwd_set_ds(void*);
int pd_flash_bwd(int, const void*, const void*, const void*, const void*, const void*, const float*, float*, void*,
                 void*, void*, float*, int, int, int, int, int, int, long, long, long, long, long, long, long, float,
                 int, void*);
}

template <typename T>
static inline T P(uintptr_t v) {
  return reinterpret_cast<T>(v);
}

static void check(int rc, const char* what) {
  if (rc != 0) throw std::runtime_error(std::string("paddle2_amd._C.") + what + " failed with code " + std::to_string(rc));
}

PYBIND11_MODULE(_C, m) {
  m.doc() = "paddle2_amd native CDNA4 (gfx950) kernels";
  m.attr("__arch__") = "gfx950";

  m.def("norm_fwd", [](int ln, int dt, int wdt, uintptr_t x, uintptr_t res, uintptr_t w, uintptr_t b, uintptr_t y,
                       uintptr_t res_out, uintptr_t mean, uintptr_t rstd, int M, int N, float eps, uintptr_t st) {
    check(pd_norm_fwd(ln, dt, wdt, P<const void*>(x), P<const void*>(res), P<const void*>(w), P<const void*>(b),
                      P<void*>(y), P<void*>(res_out), P<float*>(mean), P<float*>(rstd), M, N, eps, P<void*>(st)),
          "norm_fwd");
  });
  m.def("norm_bwd_blocks", &pd_norm_bwd_blocks);
  m.def("bias_grad_chunks", &pd_bias_grad_chunks);
  m.def("bias_grad", [](int dt, int odt, uintptr_t dy, uintptr_t part, uintptr_t db, int M, int N, uintptr_t st,
                        int acc) {
    check(pd_bias_grad(dt, odt, P<const void*>(dy), P<float*>(part), P<void*>(db), M, N, acc, P<void*>(st)),
          "bias_grad");
  }, py::arg("dt"), py::arg("odt"), py::arg("dy"), py::arg("part"), py::arg("db"), py::arg("M"), py::arg("N"),
     py::arg("st"), py::arg("acc") = 0);
  m.def("norm_bwd", [](int ln, int dt, int wdt, uintptr_t dy, uintptr_t x, uintptr_t w, uintptr_t mean, uintptr_t rstd,
                       uintptr_t dres, uintptr_t dx, uintptr_t dw_part, uintptr_t db_part, uintptr_t dw, uintptr_t db,
                       int M, int N, int nblocks, uintptr_t st, int odt, int acc_w, int acc_b) {
    check(pd_norm_bwd(ln, dt, wdt, P<const void*>(dy), P<const void*>(x), P<const void*>(w), P<const float*>(mean),
                      P<const float*>(rstd), P<const void*>(dres), P<void*>(dx), P<float*>(dw_part),
                      P<float*>(db_part), P<void*>(dw), P<void*>(db), M, N, nblocks, odt, acc_w, acc_b, P<void*>(st)),
          "norm_bwd");
  }, py::arg("ln"), py::arg("dt"), py::arg("wdt"), py::arg("dy"), py::arg("x"), py::arg("w"), py::arg("mean"),
     py::arg("rstd"), py::arg("dres"), py::arg("dx"), py::arg("dw_part"), py::arg("db_part"), py::arg("dw"),
     py::arg("db"), py::arg("M"), py::arg("N"), py::arg("nblocks"), py::arg("st"), py::arg("odt") = -1,
     py::arg("acc_w") = 0, py::arg("acc_b") = 0);
  m.def("gemm", [](int layout, int epi, uintptr_t a, long lda, uintptr_t b, long ldb, uintptr_t c, long ldc,
                   uintptr_t c2, long ldc2, uintptr_t bias, int M, int N, int K, float beta, int H, int group_m,
                   int variant, uintptr_t ws, long ws_bytes, uintptr_t st) {
    check(pd_gemm(layout, epi, P<const void*>(a), lda, P<const void*>(b), ldb, P<void*>(c), ldc, P<void*>(c2), ldc2,
                  P<const void*>(bias), M, N, K, beta, H, group_m, variant, P<void*>(ws), ws_bytes, P<void*>(st)),
          "gemm");
  });
  m.def("gemm_conv", [](uintptr_t a, long lda, uintptr_t a_lo, uintptr_t a_hi, uintptr_t b, long ldb, uintptr_t c,
                        long ldc, int M, int N, int K, int taps, int kw, int pitch, int pad_h, int pad_w, int sign,
                        int kpb_log2, int group_m, int cus, uintptr_t st) {
    return pd_gemm_conv(P<const void*>(a), lda, P<const void*>(a_lo), P<const void*>(a_hi), P<const void*>(b), ldb,
                        P<void*>(c), ldc, M, N, K, taps, kw, pitch, pad_h, pad_w, sign, kpb_log2, group_m, cus,
                        P<void*>(st));
  });
  m.def("gemm_set_rope", [](uintptr_t cos, uintptr_t sin, int cols, int seq) {
    pd_gemm_set_rope(P<const float*>(cos), P<const float*>(sin), cols, seq);
  });
  m.def("gemm_f8", [](int fa, int fb, int epi, uintptr_t a, long lda, uintptr_t b, long ldb, uintptr_t c, long ldc,
                      uintptr_t bias, uintptr_t sa, uintptr_t sb, int M, int N, int K, float beta, int group_m, int cus,
                      uintptr_t ws, long ws_bytes, uintptr_t st) {
    return pd_gemm_f8(fa, fb, epi, P<const void*>(a), lda, P<const void*>(b), ldb, P<void*>(c), ldc,
                      P<const void*>(bias), P<const float*>(sa), P<const float*>(sb), M, N, K, beta, group_m, cus,
                      P<void*>(ws), ws_bytes, P<void*>(st));
  });
  m.def("gemm_grouped", [](int layout, int epi, uintptr_t a, long lda, uintptr_t b, long ldb, long gsb, uintptr_t c,
                           long ldc, long gsc, uintptr_t c2, long ldc2, uintptr_t bias, long gsbias, uintptr_t goff,
                           int ngroups, int gmode, int M, int N, int K, int max_rows, float beta, int H, int group_m,
                           uintptr_t st) {
    check(pd_gemm_grouped(layout, epi, P<const void*>(a), lda, P<const void*>(b), ldb, gsb, P<void*>(c), ldc, gsc,
                          P<void*>(c2), ldc2, P<const void*>(bias), gsbias, P<const int*>(goff), ngroups, gmode, M, N,
                          K, max_rows, beta, H, group_m, P<void*>(st)),
          "gemm_grouped");
  });
  // ---- IPC all-reduce (csrc/kernels/ipc_allreduce.hip)
  m.def("ar_sig_bytes", []() { return pd_ar_sig_bytes(); });
  m.def("memcpy_d2d", [](uintptr_t dst, uintptr_t src, long bytes, uintptr_t st) {
    check(pd_memcpy_d2d(P<void*>(dst), P<const void*>(src), bytes, P<void*>(st)), "memcpy_d2d");
  });
  m.def("ar_alloc", [](long bytes) {
    void* p = nullptr;
    check(pd_ar_alloc(bytes, &p), "ar_alloc");
    return (uintptr_t)p;
  });
  m.def("ar_free", [](uintptr_t p) { check(pd_ar_free(P<void*>(p)), "ar_free"); });
  m.def("ar_get_handle", [](uintptr_t p) {
    char h[64];
    check(pd_ar_get_handle(P<void*>(p), h), "ar_get_handle");
    return py::bytes(h, 64);
  });
  m.def("ar_open_handle", [](py::bytes h) {
    std::string s = h;
    if (s.size() != 64) throw std::runtime_error("ar_open_handle: need a 64-byte IPC handle");
    void* p = nullptr;
    check(pd_ar_open_handle(s.data(), &p), "ar_open_handle");
    return (uintptr_t)p;
  });
  m.def("ar_close_handle", [](uintptr_t p) { check(pd_ar_close_handle(P<void*>(p)), "ar_close_handle"); });
  m.def("ar_allreduce", [](int mode, int dt, std::vector<uintptr_t> data, std::vector<uintptr_t> sig, int rank,
                           uintptr_t out, long out_stride, long bytes, long red_off, unsigned epoch, uintptr_t err,
                           int blocks, int timeout_ms, uintptr_t st) {
    if (data.size() != sig.size()) throw std::runtime_error("ar_allreduce: data/sig length mismatch");
    std::vector<const void*> d(data.size()), s(sig.size());
    for (size_t i = 0; i < data.size(); ++i) { d[i] = P<const void*>(data[i]); s[i] = P<const void*>(sig[i]); }
    check(pd_ar_allreduce(mode, dt, d.data(), s.data(), rank, (int)data.size(), P<void*>(out), out_stride, bytes,
                          red_off, epoch, P<unsigned*>(err), blocks, timeout_ms, P<void*>(st)),
          "ar_allreduce");
  });
  m.def("bias_act", [](int dt, int gated, int act, uintptr_t x, uintptr_t b, uintptr_t out, long rows, int H, long sx,
                       long so, uintptr_t st) {
    check(pd_bias_act(dt, gated, act, P<const void*>(x), P<const void*>(b), P<void*>(out), rows, H, sx, so,
                      P<void*>(st)), "bias_act");
  });
  m.def("bias_act_bwd", [](int dt, int gated, int act, uintptr_t x, uintptr_t b, uintptr_t dout, uintptr_t dx,
                           long rows, int H, long sx, long sd, uintptr_t st) {
    check(pd_bias_act_bwd(dt, gated, act, P<const void*>(x), P<const void*>(b), P<const void*>(dout), P<void*>(dx),
                          rows, H, sx, sd, P<void*>(st)), "bias_act_bwd");
  });
  m.def("dropout_add", [](int dt, int bwd, uintptr_t x, uintptr_t y, uintptr_t out, long n, unsigned seed, float p,
                          uintptr_t st) {
    check(pd_dropout_add(dt, bwd, P<const void*>(x), P<const void*>(y), P<void*>(out), n, seed, p, P<void*>(st)),
          "dropout_add");
  });
  m.def("swiglu_fwd", [](int dt, uintptr_t x, uintptr_t y, uintptr_t out, long rows, int H, long sx, long sy,
                         uintptr_t st) {
    check(pd_swiglu_fwd(dt, P<const void*>(x), P<const void*>(y), P<void*>(out), rows, H, sx, sy, P<void*>(st)),
          "swiglu_fwd");
  });
  m.def("swiglu_bwd", [](int dt, uintptr_t x, uintptr_t y, uintptr_t dout, uintptr_t dx, uintptr_t dy, long rows,
                         int H, long sx, long sy, long sdx, long sdy, uintptr_t st) {
    check(pd_swiglu_bwd(dt, P<const void*>(x), P<const void*>(y), P<const void*>(dout), P<void*>(dx), P<void*>(dy),
                        rows, H, sx, sy, sdx, sdy, P<void*>(st)),
          "swiglu_bwd");
  });
  m.def("rope", [](int dt, int style, int bwd, uintptr_t x, uintptr_t out, uintptr_t cosv, uintptr_t sinv,
                   uintptr_t pos, int B, int S, int Hn, int D, int time_major, long sx, long so, uintptr_t st) {
    check(pd_rope(dt, style, bwd, P<const void*>(x), P<void*>(out), P<const float*>(cosv), P<const float*>(sinv),
                  P<const int64_t*>(pos), B, S, Hn, D, time_major, sx, so, P<void*>(st)),
          "rope");
  });
  m.def("opt_chunk_size", &pd_opt_chunk_size);
  m.def("opt_meta_bytes", &pd_opt_meta_bytes);
  m.def("adamw_mt", [](int pdt, int gdt, int master, uintptr_t meta, uintptr_t prefix, int T, long chunks, float lr,
                       float b1, float b2, float eps, float bc1, float bc2, uintptr_t found_inf, uintptr_t inv_scale,
                       uintptr_t st) {
    check(pd_adamw_mt(pdt, gdt, master, P<const void*>(meta), P<const long*>(prefix), T, chunks, lr, b1, b2, eps, bc1,
                      bc2, P<const float*>(found_inf), P<const float*>(inv_scale), P<void*>(st)),
          "adamw_mt");
  });
  m.def("unscale_mt", [](int gdt, uintptr_t meta, uintptr_t prefix, int T, long chunks, uintptr_t scale,
                         uintptr_t found_inf, uintptr_t st) {
    check(pd_unscale_mt(gdt, P<const void*>(meta), P<const long*>(prefix), T, chunks, P<const float*>(scale),
                        P<float*>(found_inf), P<void*>(st)),
          "unscale_mt");
  });
  m.def("sqnorm_mt", [](int gdt, uintptr_t meta, uintptr_t prefix, int T, long chunks, uintptr_t out, uintptr_t st) {
    check(pd_sqnorm_mt(gdt, P<const void*>(meta), P<const long*>(prefix), T, chunks, P<float*>(out), P<void*>(st)),
          "sqnorm_mt");
  });
  m.def("scale_mt", [](int gdt, uintptr_t meta, uintptr_t prefix, int T, long chunks, uintptr_t coef, uintptr_t st) {
    check(pd_scale_mt(gdt, P<const void*>(meta), P<const long*>(prefix), T, chunks, P<const float*>(coef),
                      P<void*>(st)),
          "scale_mt");
  });
  m.def("update_loss_scaling", [](uintptr_t found_inf, uintptr_t scale, uintptr_t good, uintptr_t bad, int incr_n,
                                  int decr_n, float incr_ratio, float decr_ratio, uintptr_t st) {
    check(pd_update_loss_scaling(P<const float*>(found_inf), P<float*>(scale), P<int*>(good), P<int*>(bad), incr_n,
                                 decr_n, incr_ratio, decr_ratio, P<void*>(st)),
          "update_loss_scaling");
  });
  m.def("softmax_mask_fwd", [](int dt, int causal, uintptr_t x, uintptr_t mask, uintptr_t y, long rows, int H, int Sq,
                                int Sk, uintptr_t st) {
    check(pd_softmax_mask_fwd(dt, causal, P<const void*>(x), P<const void*>(mask), P<void*>(y), rows, H, Sq, Sk,
                              P<void*>(st)),
          "softmax_mask_fwd");
  });
  m.def("softmax_mask_bwd", [](int dt, uintptr_t y, uintptr_t dy, uintptr_t dx, long rows, int Sk, uintptr_t st) {
    check(pd_softmax_mask_bwd(dt, P<const void*>(y), P<const void*>(dy), P<void*>(dx), rows, Sk, P<void*>(st)),
          "softmax_mask_bwd");
  });
  m.def("ce_stats", [](int dt, uintptr_t logits, uintptr_t labels, uintptr_t mx, uintptr_t se, uintptr_t tgt, long N,
                       long V, long start, uintptr_t st) {
    check(pd_ce_stats(dt, P<const void*>(logits), P<const int64_t*>(labels), P<float*>(mx), P<float*>(se),
                      P<float*>(tgt), N, V, start, P<void*>(st)),
          "ce_stats");
  });
  m.def("ce_bwd", [](int dt, uintptr_t logits, uintptr_t labels, uintptr_t lse, uintptr_t dloss, uintptr_t dx, long N,
                     long V, long start, long ignore_index, int dloss_scalar, uintptr_t st) {
    check(pd_ce_bwd(dt, P<const void*>(logits), P<const int64_t*>(labels), P<const float*>(lse),
                    P<const float*>(dloss), P<void*>(dx), N, V, start, ignore_index, dloss_scalar, P<void*>(st)),
          "ce_bwd");
  });
  m.def("embed_fwd", [](int dt, uintptr_t ids, uintptr_t w, uintptr_t out, long Ntok, int H, long start, long Vl,
                        uintptr_t st) {
    check(pd_embed_fwd(dt, P<const int64_t*>(ids), P<const void*>(w), P<void*>(out), Ntok, H, start, Vl, P<void*>(st)),
          "embed_fwd");
  });
  m.def("embed_bwd", [](int dt, uintptr_t ids, uintptr_t dout, uintptr_t dw32, long Ntok, int H, long start, long Vl,
                        long padding_idx, uintptr_t st) {
    check(pd_embed_bwd(dt, P<const int64_t*>(ids), P<const void*>(dout), P<float*>(dw32), Ntok, H, start, Vl,
                       padding_idx, P<void*>(st)),
          "embed_bwd");
  });
  m.def("fp8_cast", [](int dt, int e5m2, uintptr_t x, uintptr_t y, uintptr_t yT, long R, long C, uintptr_t scale,
                       uintptr_t amax, uintptr_t st, uintptr_t colpart) {
    // colpart requested on a path without it: returns False (nothing launched) so the caller sums dY itself
    const int rc = pd_fp8_cast(dt, e5m2, P<const void*>(x), P<void*>(y), P<void*>(yT), R, C, P<const float*>(scale),
                               P<float*>(amax), P<float*>(colpart), P<void*>(st));
    if (rc == -5) return false;
    check(rc, "fp8_cast");
    return true;
  }, py::arg("dt"), py::arg("e5m2"), py::arg("x"), py::arg("y"), py::arg("yT"), py::arg("R"), py::arg("C"),
     py::arg("scale"), py::arg("amax"), py::arg("st"), py::arg("colpart") = 0);
  m.def("colsum", [](int odt, uintptr_t part, uintptr_t db, int Pn, int N, uintptr_t st, int acc) {
    check(pd_colsum(odt, P<const float*>(part), P<void*>(db), Pn, N, acc, P<void*>(st)), "colsum");
  }, py::arg("odt"), py::arg("part"), py::arg("db"), py::arg("Pn"), py::arg("N"), py::arg("st"), py::arg("acc") = 0);
  // roles: [(hist, len, amax, scale, inv, snap (0 = none), fp8_max, margin_pow2)], up to 16 in one launch
  m.def("fp8_update_scale", [](const std::vector<std::tuple<uintptr_t, int, uintptr_t, uintptr_t, uintptr_t, uintptr_t,
                                                            float, float>>& roles,
                               uintptr_t st) {
    const int n = (int)roles.size();
    std::vector<float*> hist(n), amax(n), scale(n), inv(n), snap(n);
    std::vector<int> len(n);
    std::vector<float> fmax(n), mp2(n);
    for (int i = 0; i < n; ++i) {
      const auto& r = roles[i];
      hist[i] = P<float*>(std::get<0>(r));
      len[i] = std::get<1>(r);
      amax[i] = P<float*>(std::get<2>(r));
      scale[i] = P<float*>(std::get<3>(r));
      inv[i] = P<float*>(std::get<4>(r));
      snap[i] = P<float*>(std::get<5>(r));
      fmax[i] = std::get<6>(r);
      mp2[i] = std::get<7>(r);
    }
    check(pd_fp8_update_scale(n, hist.data(), len.data(), amax.data(), scale.data(), inv.data(), snap.data(),
                              fmax.data(), mp2.data(), P<void*>(st)),
          "fp8_update_scale");
  });
  m.def("decode_attn", [](uintptr_t q, long sq_b, long sq_h, uintptr_t kc, uintptr_t vc, long s_blk, long s_tok,
                          long s_head, uintptr_t table, int max_blocks, int block_size, uintptr_t seq_lens, int max_len,
                          uintptr_t part_o, uintptr_t part_ml, uintptr_t out, long so_b, long so_h, int B, int Hq,
                          int Hk, int HD, int splits, float scale, int impl, uintptr_t st) {
    check(pd_decode_attn(P<const void*>(q), sq_b, sq_h, P<const void*>(kc), P<const void*>(vc), s_blk, s_tok, s_head,
                         P<const int*>(table), max_blocks, block_size, P<const int*>(seq_lens), max_len,
                         P<float*>(part_o), P<float*>(part_ml), P<void*>(out), so_b, so_h, B, Hq, Hk, HD, splits,
                         scale, impl, P<void*>(st)),
          "decode_attn");
  });
  m.def("cache_write", [](uintptr_t k, uintptr_t v, long sk, long sv, uintptr_t kc, uintptr_t vc, long s_blk,
                          long s_tok, long s_head, uintptr_t table, int max_blocks, int block_size, uintptr_t tok_b,
                          uintptr_t tok_p, int n_tok, int Hk, int HD, uintptr_t st) {
    check(pd_cache_write(P<const void*>(k), P<const void*>(v), sk, sv, P<void*>(kc), P<void*>(vc), s_blk, s_tok,
                         s_head, P<const int*>(table), max_blocks, block_size, P<const int*>(tok_b),
                         P<const int*>(tok_p), n_tok, Hk, HD, P<void*>(st)),
          "cache_write");
  });
  m.def("cast_from_f32", [](int dt, uintptr_t src, uintptr_t dst, long n, uintptr_t st) {
    check(pd_cast_from_f32(dt, P<const float*>(src), P<void*>(dst), n, P<void*>(st)), "cast_from_f32");
  });
  m.def("flash_bwd_block", [](int D) { return pd_flash_bwd_block(D); });
  m.def("flash_ds_elems", [](int B, int Sq, int Sk, int Hq, int D, int causal) {
    return pd_flash_ds_elems(B, Sq, Sk, Hq, D, causal);
  });
  m.def("flash_bwd_set_ds", [](uintptr_t ds) { pd_flash_bwd_set_ds(P<void*>(ds)); });
  m.def("flash_bwd_set_rope", [](uintptr_t cos, uintptr_t sin) {
    pd_flash_bwd_set_rope(P<const float*>(cos), P<const float*>(sin));
  });
  m.def("flash_fwd", [](int dt, uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t lse, int B, int Sq,
                        int Sk, int Hq, int Hk, int D, long sq_row, long sk_row, long sv_row, long so_row, float scale,
                        int causal, uintptr_t st) {
    check(pd_flash_fwd(dt, P<const void*>(q), P<const void*>(k), P<const void*>(v), P<void*>(o), P<float*>(lse), B, Sq,
                       Sk, Hq, Hk, D, sq_row, sk_row, sv_row, so_row, scale, causal, P<void*>(st)),
          "flash_fwd");
  });
  m.def("flash_bwd", [](int dt, uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t dout, uintptr_t lse,
                        uintptr_t delta, uintptr_t dq, uintptr_t dk, uintptr_t dv, uintptr_t dq32, int B, int Sq,
                        int Sk, int Hq, int Hk, int D, long sq_row, long sk_row, long sv_row, long so_row,
                        long sdq_row, long sdk_row, long sdv_row, float scale, int causal, uintptr_t st) {
    check(pd_flash_bwd(dt, P<const void*>(q), P<const void*>(k), P<const void*>(v), P<const void*>(o),
                       P<const void*>(dout), P<const float*>(lse), P<float*>(delta), P<void*>(dq), P<void*>(dk),
                       P<void*>(dv), P<float*>(dq32), B, Sq, Sk, Hq, Hk, D, sq_row, sk_row, sv_row, so_row, sdq_row,
                       sdk_row, sdv_row, scale, causal, P<void*>(st)),
          "flash_bwd");
  });
  m.def("flash_fwd_ext", [](int dt, uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t lse, int B, int Sq,
                            int Sk, int Hq, int Hk, int D, long sq_row, long sk_row, long sv_row, long so_row,
                            float scale, int causal, int mode, uintptr_t cu_q, uintptr_t cu_k, int total_q,
                            uintptr_t fm, uintptr_t fm_t64, uintptr_t fm_t256, int fm_hm, int drop, unsigned seed,
                            float pdrop, uintptr_t st) {
    check(pd_flash_fwd_ext(dt, P<const void*>(q), P<const void*>(k), P<const void*>(v), P<void*>(o), P<float*>(lse), B,
                           Sq, Sk, Hq, Hk, D, sq_row, sk_row, sv_row, so_row, scale, causal, mode,
                           P<const int*>(cu_q), P<const int*>(cu_k), total_q, P<const int*>(fm),
                           P<const int*>(fm_t64), P<const int*>(fm_t256), fm_hm, drop, seed, pdrop, P<void*>(st)),
          "flash_fwd_ext");
  });
  m.def("flash_bwd_ext", [](int dt, uintptr_t q, uintptr_t k, uintptr_t v, uintptr_t o, uintptr_t dout, uintptr_t lse,
                            uintptr_t delta, uintptr_t dq, uintptr_t dk, uintptr_t dv, uintptr_t dq32, int B, int Sq,
                            int Sk, int Hq, int Hk, int D, long sq_row, long sk_row, long sv_row, long so_row,
                            long sdq_row, long sdk_row, long sdv_row, float scale, int causal, int mode,
                            uintptr_t cu_q, uintptr_t cu_k, int total_q, uintptr_t fm, uintptr_t fm_t64,
                            uintptr_t fm_t256, int fm_hm, int drop, unsigned seed, float pdrop, uintptr_t st) {
    check(pd_flash_bwd_ext(dt, P<const void*>(q), P<const void*>(k), P<const void*>(v), P<const void*>(o),
                           P<const void*>(dout), P<const float*>(lse), P<float*>(delta), P<void*>(dq), P<void*>(dk),
                           P<void*>(dv), P<float*>(dq32), B, Sq, Sk, Hq, Hk, D, sq_row, sk_row, sv_row, so_row,
                           sdq_row, sdk_row, sdv_row, scale, causal, mode, P<const int*>(cu_q), P<const int*>(cu_k),
                           total_q, P<const int*>(fm), P<const int*>(fm_t64), P<const int*>(fm_t256), fm_hm, drop,
                           seed, pdrop, P<void*>(st)),
          "flash_bwd_ext");
  });
  m.def("transpose16", [](uintptr_t in, uintptr_t out, long M, long N, long ld_in, long ld_out, uintptr_t st) {
    check(pd_transpose16(P<const void*>(in), P<void*>(out), M, N, ld_in, ld_out, P<void*>(st)), "transpose16");
  });
  m.def("swiglu_bwd_t", [](uintptr_t x, uintptr_t g, uintptr_t dxy, uintptr_t dxyT, long M, int H, long sx,
                           uintptr_t st) {
    check(pd_swiglu_bwd_t(P<const void*>(x), P<const void*>(g), P<void*>(dxy), P<void*>(dxyT), M, H, sx, P<void*>(st)),
          "swiglu_bwd_t");
  });
  m.def("bn_workspace", &pd_bn_workspace);
  m.def("bn_fwd_train", [](int dt, uintptr_t x, uintptr_t z, uintptr_t y, long M, int C, uintptr_t rm, uintptr_t rv,
                           uintptr_t g, uintptr_t b, float momentum, float eps, uintptr_t sm, uintptr_t si,
                           uintptr_t ws, int relu, int upd, uintptr_t st) {
    check(pd_bn_fwd_train(dt, P<const void*>(x), P<const void*>(z), P<void*>(y), M, C, P<float*>(rm), P<float*>(rv),
                          P<const float*>(g), P<const float*>(b), momentum, eps, P<float*>(sm), P<float*>(si),
                          P<float*>(ws), relu, upd, P<void*>(st)),
          "bn_fwd_train");
  });
  m.def("bn_apply", [](int dt, uintptr_t x, uintptr_t z, uintptr_t y, long M, int C, uintptr_t scale, uintptr_t shift,
                       int relu, uintptr_t st) {
    check(pd_bn_apply(dt, P<const void*>(x), P<const void*>(z), P<void*>(y), M, C, P<const float*>(scale),
                      P<const float*>(shift), relu, P<void*>(st)),
          "bn_apply");
  });
  m.def("bn_bwd", [](int dt, uintptr_t dy, uintptr_t x, uintptr_t y, uintptr_t mean, uintptr_t invstd, uintptr_t g,
                     uintptr_t dx, uintptr_t dz, uintptr_t dg, uintptr_t db, long M, int C, uintptr_t ws, int relu,
                     uintptr_t st) {
    check(pd_bn_bwd(dt, P<const void*>(dy), P<const void*>(x), P<const void*>(y), P<const float*>(mean),
                    P<const float*>(invstd), P<const float*>(g), P<void*>(dx), P<void*>(dz), P<float*>(dg),
                    P<float*>(db), M, C, P<float*>(ws), relu, P<void*>(st)),
          "bn_bwd");
  });
  m.def("dec_splits", &pd_dec_splits);
  m.def("dec64_gemm", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t out, int M, int N, int K, int kw,
                         int rt, uintptr_t st) {
    check(pd_dec64_gemm(P<const void*>(x), P<const void*>(w), P<const void*>(bias), P<void*>(out), M, N, K, kw, rt,
                        P<void*>(st)),
          "dec64_gemm");
  });
  m.def("dec64_rt", &pd_dec64_rt);
  m.def("dec64s_gemm", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t out, uintptr_t ws, int M, int N, int K,
                          int dw, int rt, int S, uintptr_t st) {
    check(pd_dec64s_gemm(P<const void*>(x), P<const void*>(w), P<const void*>(bias), P<void*>(out), P<float*>(ws), M,
                         N, K, dw, rt, S, P<void*>(st)),
          "dec64s_gemm");
  });
  m.def("dec64s_workspace", &pd_dec64s_workspace);
  m.def("dec_gemm", [](uintptr_t x, uintptr_t w, uintptr_t bias, uintptr_t out, uintptr_t ws, int M, int N, int K,
                       int S, uintptr_t st, int glu, uintptr_t cnt, int noreduce) {
    check(pd_dec_gemm(P<const void*>(x), P<const void*>(w), P<const void*>(bias), P<void*>(out), P<float*>(ws), M, N,
                      K, S, glu, P<int*>(cnt), P<void*>(st), noreduce),
          "dec_gemm");
  }, py::arg("x"), py::arg("w"), py::arg("bias"), py::arg("out"), py::arg("ws"), py::arg("M"), py::arg("N"),
     py::arg("K"), py::arg("S"), py::arg("st"), py::arg("glu") = 0, py::arg("cnt") = 0, py::arg("noreduce") = 0);
  m.def("dec_reduce", [](uintptr_t ws, int S, int M, int N, uintptr_t bias, uintptr_t out, uintptr_t st) {
    check(pd_dec_reduce(P<const float*>(ws), S, M, N, P<const void*>(bias), P<void*>(out), P<void*>(st)), "dec_reduce");
  });
  m.def("norm_fwd_part", [](int wdt, uintptr_t part, int S, uintptr_t res, uintptr_t w, uintptr_t y, uintptr_t res_out,
                            int M, int N, float eps, uintptr_t st) {
    check(pd_norm_fwd_part(wdt, P<const float*>(part), S, P<const void*>(res), P<const void*>(w), P<void*>(y),
                           P<void*>(res_out), M, N, eps, P<void*>(st)),
          "norm_fwd_part");
  });
  m.def("wo_splits", &pd_wo_splits);
  m.def("wo_workspace", &pd_wo_workspace);
  m.def("wo_gemm", [](int int4, uintptr_t x, uintptr_t w, uintptr_t cs, uintptr_t gs, int group, uintptr_t bias,
                      uintptr_t out, uintptr_t ws, int M, int N, int K, int S, uintptr_t st) {
    check(pd_wo_gemm(int4, P<const void*>(x), P<const void*>(w), P<const float*>(cs), P<const float*>(gs), group,
                     P<const void*>(bias), P<void*>(out), P<float*>(ws), M, N, K, S, P<void*>(st)),
          "wo_gemm");
  });
}
