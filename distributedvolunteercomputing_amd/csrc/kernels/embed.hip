// Token (+ position) embedding forward/backward for gfx950.
//
// fwd: x[r, :] = wte[idx[r], :] (+ wpe[r % T, :])  — 16-B row gathers, one wave per row
// bwd: token table: dwte[idx[r], :] += dx[r, :] with fp32 global atomics into a zeroed scratch
//      (each wave-instruction adds 256 contiguous bytes: the full-rate atomic shape), then one
//      pass that adds the scratch into the bf16 gradient (the flat .grad view when given).
//      position table: dwpe[t, :] = sum_b dx[b, t, :] is a plain column reduction over the batch
//      (no atomics: all B rows of one position are summed by one thread).
// Unlike torch's sort/segment-based embedding backward (data-dependent partition kernels),
// this is graph-capture safe: fixed launch shapes, no host round trip, no dynamic sizes.
#include "vcx_common.h"

namespace vcx {

__global__ void __launch_bounds__(256) embed_fwd_kernel(const int64_t* __restrict__ idx, const bf16* __restrict__ wte,
                                                         const bf16* __restrict__ wpe, bf16* __restrict__ out,
                                                         int64_t R, int T, int C, int V) {
  const int lane = threadIdx.x & 63;
  const int C8 = C >> 3;
  for (int64_t r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < R; r += (int64_t)gridDim.x * 4) {
    int64_t t = idx[r];
    t = t < 0 ? 0 : (t >= V ? V - 1 : t);  // clamp: never gather out of bounds
    const bf16* src = wte + t * C;
    const bf16* pos = wpe ? wpe + (int64_t)(r % T) * C : nullptr;
    for (int c = lane; c < C8; c += 64) {
      bf16x8 v = *(const bf16x8*)(src + c * 8);
      if (pos) {
        bf16x8 p = *(const bf16x8*)(pos + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] + (float)p[j]);
      }
      *(bf16x8*)(out + r * C + c * 8) = v;
    }
  }
}

// one wave per token row; lane l adds columns l, l + 64, ... (256 contiguous bytes per atomic
// wave-instruction); the row's bf16 loads are issued before its atomics
template <int CPL>
__global__ void __launch_bounds__(256) embed_bwd_tok_kernel(const int64_t* __restrict__ idx,
                                                             const bf16* __restrict__ dx, float* __restrict__ dwte,
                                                             int64_t R, int C, int V) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < R; r += (int64_t)gridDim.x * 4) {
    const int64_t t = idx[r];
    if (t < 0 || t >= V) continue;
    const bf16* src = dx + r * C;
    float* dst = dwte + t * C;
    float v[CPL];
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      v[k] = c < C ? (float)src[c] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < CPL; ++k) {
      const int c = lane + 64 * k;
      if (c < C) atomicAdd(dst + c, v[k]);
    }
  }
}

// dwpe[t, c8] (+)= sum over the batch of dx[b, t, c8]; rows t >= T of dwpe are left untouched
__global__ void __launch_bounds__(256) embed_bwd_pos_kernel(const bf16* __restrict__ dx, bf16* __restrict__ dwpe,
                                                             int Bn, int T, int C, int accumulate) {
  const int C8 = C >> 3;
  const int64_t n = (int64_t)T * C8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int t = (int)(i / C8), c8 = (int)(i % C8);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int b = 0;
    for (; b + 3 < Bn; b += 4) {
      bf16x8 v[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = *(const bf16x8*)(dx + ((int64_t)(b + u) * T + t) * C + c8 * 8);
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += (float)v[u][j];
    }
    for (; b < Bn; ++b) {
      bf16x8 v = *(const bf16x8*)(dx + ((int64_t)b * T + t) * C + c8 * 8);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
    }
    bf16* o = dwpe + (int64_t)t * C + c8 * 8;
    bf16x8 out;
    if (accumulate) {
      bf16x8 old = *(const bf16x8*)o;
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = (bf16)(acc[j] + (float)old[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) out[j] = (bf16)acc[j];
    }
    *(bf16x8*)o = out;
  }
}

// acc(bf16) (+)= src(f32), 8 elements per lane
__global__ void __launch_bounds__(256) f32_into_bf16_kernel(const float* __restrict__ src, bf16* __restrict__ acc,
                                                             int64_t n8, int accumulate) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t b = i * 8;
    f32x4 a0 = *(const f32x4*)(src + b), a1 = *(const f32x4*)(src + b + 4);
    float f[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    bf16x8 o;
    if (accumulate) {
      bf16x8 old = *(const bf16x8*)(acc + b);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)(f[j] + (float)old[j]);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)f[j];
    }
    *(bf16x8*)(acc + b) = o;
  }
}

}  // namespace vcx

using namespace vcx;

void vcx_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int64_t R, int T, int C, int V,
                   hipStream_t s) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(stream_grid(R, 4, 4096)), dim3(256), 0, s, idx, (const bf16*)wte,
                     (const bf16*)wpe, (bf16*)out, R, T, C, V);
}

void vcx_embed_bwd(const int64_t* idx, const void* dx, float* dwte_scratch, void* dwte, int accum_wte, void* dwpe,
                   int accum_wpe, int64_t R, int T, int C, int V, hipStream_t s) {
  const dim3 g(stream_grid(R, 4, 4096));
  const int cpl = (C + 63) / 64;
  if (cpl <= 12)
    hipLaunchKernelGGL(embed_bwd_tok_kernel<12>, g, dim3(256), 0, s, idx, (const bf16*)dx, dwte_scratch, R, C, V);
  else if (cpl <= 32)
    hipLaunchKernelGGL(embed_bwd_tok_kernel<32>, g, dim3(256), 0, s, idx, (const bf16*)dx, dwte_scratch, R, C, V);
  else
    hipLaunchKernelGGL(embed_bwd_tok_kernel<128>, g, dim3(256), 0, s, idx, (const bf16*)dx, dwte_scratch, R, C, V);
  const int64_t n8 = (int64_t)V * C / 8;
  hipLaunchKernelGGL(f32_into_bf16_kernel, dim3(stream_grid(n8, 256)), dim3(256), 0, s, dwte_scratch, (bf16*)dwte, n8,
                     accum_wte);
  if (dwpe) {
    const int64_t np = (int64_t)T * (C / 8);
    hipLaunchKernelGGL(embed_bwd_pos_kernel, dim3(stream_grid(np, 256)), dim3(256), 0, s, (const bf16*)dx,
                       (bf16*)dwpe, (int)(R / T), T, C, accum_wpe);
  }
}
