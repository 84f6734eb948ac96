// Host-side launcher declarations for every gfx950 kernel of the package. Kernel files
// (*.hip, built by hipcc --offload-arch=gfx950) define them; the torch bindings call them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

// optim.hip
void vcx_grad_sumsq(const void* g, int64_t n, float* ostate, hipStream_t s);
void vcx_adam_prologue(float* ostate, float max_norm, hipStream_t s);
void vcx_adamw_flat(void* param, const void* grad, float* master, float* m, float* v, int64_t n, int64_t n_decay,
                    const float* ostate, float beta1, float beta2, float eps, float wd, hipStream_t s);
void vcx_lsgd_delta(const float* master, const float* anchor, void* delta, int64_t n, hipStream_t s);
void vcx_lsgd_apply(const void* avg, float* anchor, float* master, void* param, float* mom, int64_t n,
                    float outer_lr, float mu, int nesterov, float avg_scale, hipStream_t s);
void vcx_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t s);
void vcx_axpy_bf16(const void* src, void* acc, int64_t n, float scale, hipStream_t s);
// gemm_wg.hip: weight gradient out (+)= A[K, M]^T B[K, N] (token-major operands), split-K fp32 partials
bool vcx_gemm_wg_supported(int M, int N, int K, int splits);
int vcx_gemm_wg_splits(int M, int N, int K);
void vcx_gemm_wg(const void* A, const void* B, float* Cpart, void* out, int M, int N, int K, int lda, int ldb,
                 int splits, int accumulate, int loaders, hipStream_t s);
bool vcx_gemm_wg_conv3x3_supported(int Cout, int Cin, int tokens, int64_t xbytes, int splits);
void vcx_gemm_wg_conv3x3(const void* dy, const void* x, float* Cpart, void* out, int Cout, int Cin, int imgs, int H,
                         int W, int stride, int splits, int accumulate, hipStream_t s);
// gemm_f.hip: C[M, N] = A[M, K] B[N, K]^T (+ bias[N]), 4 waves of 128 x 128 (the library's forward geometry)
bool vcx_gemm_f_supported(int M, int N, int K);
bool vcx_gemm_f_split_ok(int M, int N, int K, int splits);
int vcx_gemm_f_splits(int M, int N, int K);
void vcx_gemm_f(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda, int ldb,
                int ldc, int waves, int splits, float* ws, hipStream_t s);
bool vcx_gemm_f_conv3x3_supported(int imgs, int H, int W, int Cin, int Cout, int stride);
void vcx_gemm_f_conv3x3(const void* x, const void* w, void* y, const void* bias, int imgs, int H, int W, int Cin,
                        int Cout, int stride, int waves, int splits, float* ws, int flip, int tap_major,
                        hipStream_t s);
bool vcx_gemm_nt_supported(int M, int N, int K);
bool vcx_gemm_nt_supported_epi(int M, int N, int K, int epi);
void vcx_gemm_nt(const void* A, const void* B, void* C, void* C2, const void* bias, float* colsum, int M, int N, int K,
                 int lda, int ldb, int ldc, int epi, hipStream_t s);
// gemm_ps.hip: persistent store-overlapped GEMM, C = A B^T (B [N, K]); epi 0 store, 1 +bias,
// 2 +bias -> (C = pre, C2 = gelu(pre)); grid_cap <= 0: one workgroup per CU
bool vcx_gemm_ps_supported(int M, int N, int K, int epi);
int vcx_gemm_ps_grid(int M, int N, int grid_cap);
// epi 4: C = (A B^T) * gelu'(C2) with fp32 column sums added into colsum
void vcx_gemm_ps(const void* A, const void* B, void* C, void* C2, const void* bias, float* colsum, int M, int N,
                 int K, int lda, int ldb, int ldc, int epi, int grid_cap, hipStream_t s);
void vcx_transpose_bf16(const void* src, void* dst, int R, int Cc, hipStream_t s);
void vcx_add_f32_into_bf16(float* in, void* out, int n, int accumulate, int zero_in, hipStream_t s);
void vcx_reduce_bcast_bf16(const void* in, void* out, void* mine, int P, int64_t n, hipStream_t s);
void vcx_splitk_reduce(const void* part, void* acc, int S, int64_t n, int accumulate, hipStream_t s);

// norm_act.hip
void vcx_ln_fwd(const void* a, const void* b, void* xout, void* y, const void* w, const void* bias, float* mean,
                float* rstd, int R, int C, float eps, int rms, const void* bb, hipStream_t s);
int vcx_bias_gelu_partials(int R);
void vcx_bias_gelu_fwd(const void* x, const void* b, void* y, int R, int F, hipStream_t s);
constexpr int VCX_COLSUM_NB = 32;  // stage-1 row chunks of the two-stage column sums (stage: 3 * NB * C fp32)
void vcx_bias_gelu_bwd(const void* x, const void* b, const void* dy, void* dx, float* part, void* db, int R, int F,
                       float* stage, int accumulate, hipStream_t s);
// column sums of a bf16 [R, F] matrix into out[F] (bf16; added to it when accumulate != 0)
// out[C] (+)= column sums of fp32 partial rows part[P, C] (bf16 out; stage: VCX_COLSUM_NB * C fp32)
void vcx_colsum_f32(const float* part, void* out, int P, int C, int accumulate, float* stage, hipStream_t s);
void vcx_colsum_bf16(const void* y, float* part, void* out, int R, int F, int accumulate, float* stage,
                     hipStream_t s);
int vcx_ln_bwd_partials(int R, int C);
void vcx_ln_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, const void* dres,
                void* dx, float* dw_part, float* db_part, void* dw, void* db, int R, int C, int rms, float* dbb_part,
                void* dbb, float* stage, int accum_mask, hipStream_t s);
void vcx_gelu_fwd(const void* x, void* y, int64_t n, hipStream_t s);
void vcx_gelu_bwd(const void* x, const void* dy, void* dx, int64_t n, hipStream_t s);
void vcx_swiglu_fwd(const void* gu, void* y, int64_t R, int F, hipStream_t s);
void vcx_swiglu_bwd(const void* gu, const void* dy, void* dgu, int64_t R, int F, hipStream_t s);
void vcx_xent_fwd(const void* logits, const int64_t* tgt, float* lse, float* loss, int64_t R, int V, int Vp,
                  hipStream_t s);
int vcx_xent_fused(void* logits, const int64_t* tgt, const float* nvalid, float* loss, int64_t R, int V, int Vp,
                   hipStream_t s);
void vcx_xent_rescale(void* d, const float* dloss, int64_t n, hipStream_t s);
void vcx_xent_bwd(const void* logits, const int64_t* tgt, const float* lse, const float* gscale, void* dlogits,
                  int64_t R, int V, int Vp, hipStream_t s);

// attention.hip (causal flash attention, head dim 64, packed qkv)
void vcx_attn_fwd_d64(const void* qkv, void* out, float* lse, int B, int T, int H, float scale, hipStream_t s);
// variants: forward 2 or 3 waves per SIMD (default 3); K/V (Q/dO) tile staging through registers
// (0) or LDS-DMA (1) for the forward (default 1) and the backward (bit 0: dQ, bit 1: dK/dV; default 1)
void vcx_attn_set_variant(int fwd_wpe, int fwd_dma, int bwd_dma, int stage_epi);  // stage_epi: LDS-staged output stores (-1 = unchanged)
// bias_part (nullable): [B * ceil(T/128), 3 * H * 64] fp32, one row of column sums of dqkv per
// 128-row block (the gradient of a bias added to qkv: reduce with vcx_colsum_f32)
void vcx_attn_bwd_d64(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv,
                      float* bias_part, int B, int T, int H, float scale, hipStream_t s);
int vcx_attn_bias_partials(int B, int T);
// attention_hm.hip (causal flash attention, head-major GQA layout, head dim 64 or 128):
// q [B, Hq, T, D], k / v [B, Hkv, T, D], out / dout [B, T, Hq, D], lse / delta [B, Hq, T] fp32,
// dq [B, Hq, T, D], dk / dv [B, Hkv, T, D]
void vcx_attn_hm_fwd(const void* q, const void* k, const void* v, void* out, float* lse, int B, int T, int Hq, int Hkv,
                     int D, float scale, hipStream_t s);
void vcx_attn_hm_set_variant(int dkv_split);  // D = 128: 1 = dK and dV in two launches, 0 = one
void vcx_attn_hm_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout, const float* lse,
                     float* delta, void* dq, void* dk, void* dv, int B, int T, int Hq, int Hkv, int D, float scale,
                     hipStream_t s);

// rope.hip: rotary embedding fused with the QKV split into head-major q/k/v (and its inverse)
void vcx_rope_qkv(void* qkv, void* q, void* k, void* v, const float* cosv, const float* sinv, int B, int T, int Hq,
                  int Hkv, int D, int backward, hipStream_t s);

// embed.hip
void vcx_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int64_t R, int T, int C, int V,
                   hipStream_t s);
// dwte (+)= scatter of dx over idx (fp32 atomics into the zeroed dwte_scratch, then added into the
// bf16 dwte); dwpe (+)= per-position sums of dx over the batch (nullptr: no position table)
void vcx_embed_bwd(const int64_t* idx, const void* dx, float* dwte_scratch, void* dwte, int accum_wte, void* dwpe,
                   int accum_wpe, int64_t R, int T, int C, int V, hipStream_t s);
// batchnorm.hip: train-mode BatchNorm (+ residual) (+ ReLU), NHWC bf16 [R, C]
bool vcx_bn_supported(int C);
void vcx_bn_fwd_train(const void* x, const void* res, void* y, void* mask, int64_t R, int C, const void* gamma,
                      const void* beta, void* run_mean, void* run_var, int run_fp32, float eps, float momentum, float* ws,
                      float* mean, float* rstd, float* scale, float* shift, int64_t* nbt, int relu, int layer_ws,
                      hipStream_t s);
void vcx_subsample_nhwc(const void* x, void* y, int N, int H, int W, int C, int s, hipStream_t st);
void vcx_subsample_add_nhwc(void* full, const void* g, int N, int H, int W, int C, int s, hipStream_t st);
void vcx_bcast_hw_nhwc(const void* g, void* out, int N, int HW, int C, float scale, hipStream_t st);
void vcx_maxpool3s2_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int OH, int OW, hipStream_t s);
void vcx_maxpool3s2_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int OH, int OW,
                        hipStream_t s);
void vcx_bn_apply(const void* x, const void* res, void* y, int64_t R, int C, const float* scale, const float* shift,
                  int relu, hipStream_t s);
void vcx_bn_bwd(const void* dy, const void* mask, const void* x, const float* mean, const float* rstd, const float* scale,
                int64_t R, int C, float* ws, float* sums, void* gw, void* gb, void* dx, void* dres, int relu,
                int layer_ws, hipStream_t s);
