// Token (+ position) embedding forward/backward for gfx950.
//
// fwd: x[r, :] = wte[idx[r], :] (+ wpe[r % T, :])  — 16-B row gathers, one wave per row
// bwd: dwte[idx[r], :] += dx[r, :]  (+ dwpe[r % T, :] += dx[r, :]) with fp32 global atomics into
//      a zeroed scratch, then one conversion pass to the bf16 gradient.
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

__global__ void __launch_bounds__(256) embed_bwd_kernel(const int64_t* __restrict__ idx, const bf16* __restrict__ dx,
                                                         float* __restrict__ dwte, float* __restrict__ dwpe,
                                                         int64_t R, int T, int C, int V) {
  const int lane = threadIdx.x & 63;
  for (int64_t r = blockIdx.x * 4ll + (threadIdx.x >> 6); r < R; r += (int64_t)gridDim.x * 4) {
    int64_t t = idx[r];
    if (t < 0 || t >= V) continue;
    float* dst = dwte + t * C;
    float* pdst = dwpe ? dwpe + (int64_t)(r % T) * C : nullptr;
    // each lane adds 2 consecutive floats per step: 64 lanes x 8 B = one 512-B row segment
    for (int c = lane * 2; c < C; c += 128) {
      const float a = (float)dx[r * C + c], b = (float)dx[r * C + c + 1];
      atomicAdd(dst + c, a);
      atomicAdd(dst + c + 1, b);
      if (pdst) {
        atomicAdd(pdst + c, a);
        atomicAdd(pdst + c + 1, b);
      }
    }
  }
}

}  // namespace vcx

using namespace vcx;

void vcx_embed_fwd(const int64_t* idx, const void* wte, const void* wpe, void* out, int64_t R, int T, int C, int V,
                   hipStream_t s) {
  hipLaunchKernelGGL(embed_fwd_kernel, dim3(stream_grid(R, 4, 4096)), dim3(256), 0, s, idx, (const bf16*)wte,
                     (const bf16*)wpe, (bf16*)out, R, T, C, V);
}

void vcx_embed_bwd(const int64_t* idx, const void* dx, float* dwte, float* dwpe, int64_t R, int T, int C, int V,
                   hipStream_t s) {
  hipLaunchKernelGGL(embed_bwd_kernel, dim3(stream_grid(R, 4, 4096)), dim3(256), 0, s, idx, (const bf16*)dx, dwte,
                     dwpe, R, T, C, V);
}
