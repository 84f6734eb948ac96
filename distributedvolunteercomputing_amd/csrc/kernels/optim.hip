// Fused optimizer + local-SGD synchronisation kernels (gfx950).
//
// The trainer keeps every parameter of a model in ONE flat bf16 buffer (compute copy),
// with fp32 master weights, fp32 Adam moments and a bf16 flat gradient buffer of the same
// length. That turns "multi-tensor apply" into a single streaming kernel over contiguous
// memory (16 B per lane per access) and lets the local-SGD averaging move one buffer.
//
// Graph-safety: nothing here reads a host scalar that changes per step. The optimizer
// state block `ostate` (fp32, device) holds {step, lr, clip_coef, sumsq}; a 1-thread
// prologue kernel advances `step` and derives `clip_coef` from the gradient sum of squares,
// so a captured hipGraph replays a correct AdamW step every time.
//
// No reference analog ("Fused Adam (HIP)"; BASELINE.json north_star).
#include "vcx_common.h"

namespace vcx {

enum OState { OS_STEP = 0, OS_LR = 1, OS_CLIP = 2, OS_SUMSQ = 3, OS_NUM = 4 };

// ---------------------------------------------------------------- grad sum of squares
__global__ void __launch_bounds__(256) grad_sumsq_kernel(const bf16* __restrict__ g, int64_t n8,
                                                          float* __restrict__ ostate) {
  __shared__ float scratch[4];
  float acc = 0.f;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    bf16x8 v = *(const bf16x8*)(g + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float f = (float)v[j];
      acc = fmaf(f, f, acc);
    }
  }
  float s = block_sum<256>(acc, scratch);
  if (threadIdx.x == 0) atomicAdd(ostate + OS_SUMSQ, s);
}

// step += 1 ; clip_coef = min(1, max_norm / (||g|| + 1e-6))   (max_norm <= 0: no clipping)
__global__ void adam_prologue_kernel(float* __restrict__ ostate, float max_norm) {
  if (threadIdx.x == 0) {
    ostate[OS_STEP] += 1.f;
    float coef = 1.f;
    if (max_norm > 0.f) {
      float nrm = sqrtf(ostate[OS_SUMSQ]);
      coef = fminf(1.f, max_norm / (nrm + 1e-6f));
    }
    ostate[OS_CLIP] = coef;
  }
}

// AdamW over [0, n): elements [0, n_decay) get decoupled weight decay, the rest do not.
// param(bf16) <- bf16(master);  master, m, v updated in fp32.
__global__ void __launch_bounds__(256) adamw_flat_kernel(bf16* __restrict__ param, const bf16* __restrict__ grad,
                                                          float* __restrict__ master, float* __restrict__ m,
                                                          float* __restrict__ v, int64_t n8, int64_t n_decay,
                                                          const float* __restrict__ ostate, float beta1,
                                                          float beta2, float eps, float wd) {
  const float step = ostate[OS_STEP];
  const float lr = ostate[OS_LR];
  const float clip = ostate[OS_CLIP];
  const float bc1 = 1.f - powf(beta1, step);
  const float bc2 = 1.f - powf(beta2, step);
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = rsqrtf(bc2);
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t base = i * 8;
    bf16x8 gv = *(const bf16x8*)(grad + base);
    f32x4 w0 = *(const f32x4*)(master + base), w1 = *(const f32x4*)(master + base + 4);
    f32x4 m0 = *(const f32x4*)(m + base), m1 = *(const f32x4*)(m + base + 4);
    f32x4 v0 = *(const f32x4*)(v + base), v1 = *(const f32x4*)(v + base + 4);
    const float decay = (base < n_decay) ? (1.f - lr * wd) : 1.f;
    float w[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
    float mm[8] = {m0[0], m0[1], m0[2], m0[3], m1[0], m1[1], m1[2], m1[3]};
    float vv[8] = {v0[0], v0[1], v0[2], v0[3], v1[0], v1[1], v1[2], v1[3]};
    bf16x8 pout;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gj = (float)gv[j] * clip;
      mm[j] = fmaf(beta1, mm[j], (1.f - beta1) * gj);
      vv[j] = fmaf(beta2, vv[j], (1.f - beta2) * gj * gj);
      float denom = sqrtf(vv[j]) * inv_sqrt_bc2 + eps;
      w[j] = w[j] * decay - step_size * (mm[j] / denom);
      pout[j] = (bf16)w[j];
    }
    *(f32x4*)(master + base) = f32x4{w[0], w[1], w[2], w[3]};
    *(f32x4*)(master + base + 4) = f32x4{w[4], w[5], w[6], w[7]};
    *(f32x4*)(m + base) = f32x4{mm[0], mm[1], mm[2], mm[3]};
    *(f32x4*)(m + base + 4) = f32x4{mm[4], mm[5], mm[6], mm[7]};
    *(f32x4*)(v + base) = f32x4{vv[0], vv[1], vv[2], vv[3]};
    *(f32x4*)(v + base + 4) = f32x4{vv[4], vv[5], vv[6], vv[7]};
    *(bf16x8*)(param + base) = pout;
  }
}

// ---------------------------------------------------------------- local-SGD sync
// delta = bf16(master - anchor): the "pseudo-gradient" each peer contributes to the average.
__global__ void __launch_bounds__(256) lsgd_delta_kernel(const float* __restrict__ master,
                                                          const float* __restrict__ anchor,
                                                          bf16* __restrict__ delta, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    f32x4 a0 = *(const f32x4*)(master + b), a1 = *(const f32x4*)(master + b + 4);
    f32x4 c0 = *(const f32x4*)(anchor + b), c1 = *(const f32x4*)(anchor + b + 4);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (bf16)(a0[j] - c0[j]);
      o[j + 4] = (bf16)(a1[j] - c1[j]);
    }
    *(bf16x8*)(delta + b) = o;
  }
}

// Outer step after the all-reduce. avg = mean over live peers of delta (already divided).
//   pseudo-grad g = -avg ; mom = mu*mom + g ; upd = nesterov ? g + mu*mom : mom
//   anchor -= outer_lr * upd ; master = anchor ; param = bf16(anchor)
// With outer_lr = 1, mu = 0 this is plain model averaging (classic local SGD).
__global__ void __launch_bounds__(256) lsgd_apply_kernel(const bf16* __restrict__ avg, float* __restrict__ anchor,
                                                          float* __restrict__ master, bf16* __restrict__ param,
                                                          float* __restrict__ mom, int64_t n8, float outer_lr,
                                                          float mu, int nesterov, float avg_scale) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    bf16x8 d = *(const bf16x8*)(avg + b);
    f32x4 a0 = *(const f32x4*)(anchor + b), a1 = *(const f32x4*)(anchor + b + 4);
    float a[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    float mo[8];
    if (mom) {
      f32x4 q0 = *(const f32x4*)(mom + b), q1 = *(const f32x4*)(mom + b + 4);
      mo[0] = q0[0]; mo[1] = q0[1]; mo[2] = q0[2]; mo[3] = q0[3];
      mo[4] = q1[0]; mo[5] = q1[1]; mo[6] = q1[2]; mo[7] = q1[3];
    }
    bf16x8 p;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float g = -(float)d[j] * avg_scale;
      float upd = g;
      if (mom) {
        mo[j] = fmaf(mu, mo[j], g);
        upd = nesterov ? fmaf(mu, mo[j], g) : mo[j];
      }
      a[j] = fmaf(-outer_lr, upd, a[j]);
      p[j] = (bf16)a[j];
    }
    f32x4 o0 = {a[0], a[1], a[2], a[3]}, o1 = {a[4], a[5], a[6], a[7]};
    *(f32x4*)(anchor + b) = o0;
    *(f32x4*)(anchor + b + 4) = o1;
    *(f32x4*)(master + b) = o0;
    *(f32x4*)(master + b + 4) = o1;
    *(bf16x8*)(param + b) = p;
    if (mom) {
      *(f32x4*)(mom + b) = f32x4{mo[0], mo[1], mo[2], mo[3]};
      *(f32x4*)(mom + b + 4) = f32x4{mo[4], mo[5], mo[6], mo[7]};
    }
  }
}

// dst(bf16) = bf16(src(f32)) — used after checkpoint restore / re-shard.
__global__ void __launch_bounds__(256) f32_to_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ dst,
                                                           int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    f32x4 a0 = *(const f32x4*)(src + b), a1 = *(const f32x4*)(src + b + 4);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      o[j] = (bf16)a0[j];
      o[j + 4] = (bf16)a1[j];
    }
    *(bf16x8*)(dst + b) = o;
  }
}

// acc(f32) += scale * src(bf16)  — reduction step used by the hand-rolled butterfly/ring
// all-reduce (received half-buffer summed into the local accumulator).
__global__ void __launch_bounds__(256) axpy_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ acc,
                                                         int64_t n8, float scale) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    bf16x8 s = *(const bf16x8*)(src + b);
    bf16x8 a = *(const bf16x8*)(acc + b);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)fmaf(scale, (float)s[j], (float)a[j]);
    *(bf16x8*)(acc + b) = o;
  }
}

// acc[i] (+)= sum_s part[s * n + i]: the split-M weight-gradient reduction. The S partial
// products come from ONE batched GEMM over S token chunks (more output tiles in flight than the
// single K = tokens GEMM); they are summed in fp32 straight into the flat gradient buffer.
__global__ void __launch_bounds__(256) splitk_reduce_kernel(const bf16* __restrict__ part, bf16* __restrict__ acc,
                                                            int S, int64_t n8, int accumulate) {
  const int64_t n = n8 * 8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    float t[8];
    if (accumulate) {
      bf16x8 a = *(const bf16x8*)(acc + b);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = (float)a[j];
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] = 0.f;
    }
    for (int k = 0; k < S; ++k) {
      bf16x8 v = *(const bf16x8*)(part + k * n + b);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] += (float)v[j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)t[j];
    *(bf16x8*)(acc + b) = o;
  }
}

}  // namespace vcx

// ---------------------------------------------------------------- launchers
using namespace vcx;

void vcx_grad_sumsq(const void* g, int64_t n, float* ostate, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(grad_sumsq_kernel, dim3(stream_grid(n8, 256, 1024)), dim3(256), 0, s, (const bf16*)g, n8,
                     ostate);
}

void vcx_adam_prologue(float* ostate, float max_norm, hipStream_t s) {
  hipLaunchKernelGGL(adam_prologue_kernel, dim3(1), dim3(64), 0, s, ostate, max_norm);
}

void vcx_adamw_flat(void* param, const void* grad, float* master, float* m, float* v, int64_t n, int64_t n_decay,
                    const float* ostate, float beta1, float beta2, float eps, float wd, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(adamw_flat_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, (bf16*)param,
                     (const bf16*)grad, master, m, v, n8, n_decay, ostate, beta1, beta2, eps, wd);
}

void vcx_lsgd_delta(const float* master, const float* anchor, void* delta, int64_t n, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(lsgd_delta_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, master, anchor,
                     (bf16*)delta, n8);
}

void vcx_lsgd_apply(const void* avg, float* anchor, float* master, void* param, float* mom, int64_t n,
                    float outer_lr, float mu, int nesterov, float avg_scale, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(lsgd_apply_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, (const bf16*)avg, anchor,
                     master, (bf16*)param, mom, n8, outer_lr, mu, nesterov, avg_scale);
}

void vcx_f32_to_bf16(const float* src, void* dst, int64_t n, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(f32_to_bf16_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, src, (bf16*)dst, n8);
}

// Direct all-reduce, middle step: this peer received its shard from all P peers (rows of
// `in`, row stride n); sum them in fp32 and write the sum to all P rows of `out` (the send
// buffer of the all-gather all-to-all, one row per destination) and to `mine` (this peer's
// shard of the averaged buffer). One pass: reads P*n, writes (P+1)*n bf16.
__global__ void __launch_bounds__(256) reduce_bcast_bf16_kernel(const bf16* __restrict__ in, bf16* __restrict__ out,
                                                               bf16* __restrict__ mine, int P, int64_t n8) {
  const int64_t n = n8 * 8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    float t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = 0.f;
    for (int k = 0; k < P; ++k) {
      bf16x8 v = *(const bf16x8*)(in + k * n + b);
#pragma unroll
      for (int j = 0; j < 8; ++j) t[j] += (float)v[j];
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)t[j];
    if (out)
      for (int k = 0; k < P; ++k) *(bf16x8*)(out + k * n + b) = o;
    if (mine) *(bf16x8*)(mine + b) = o;
  }
}

void vcx_reduce_bcast_bf16(const void* in, void* out, void* mine, int P, int64_t n, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(reduce_bcast_bf16_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, (const bf16*)in,
                     (bf16*)out, (bf16*)mine, P, n8);
}

void vcx_axpy_bf16(const void* src, void* acc, int64_t n, float scale, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(axpy_bf16_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, (const bf16*)src,
                     (bf16*)acc, n8, scale);
}

void vcx_splitk_reduce(const void* part, void* acc, int S, int64_t n, int accumulate, hipStream_t s) {
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(splitk_reduce_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, (const bf16*)part,
                     (bf16*)acc, S, n8, accumulate);
}
