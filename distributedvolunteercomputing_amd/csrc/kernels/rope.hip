// Rotary position embedding fused with the QKV split / head-major relayout (Llama-3 attention).
//
// fwd: qkv [B, T, (Hq + 2 Hkv) * D] (the fused QKV projection output, token-major)
//      -> q [B, Hq, T, D], k [B, Hkv, T, D] rotated, v [B, Hkv, T, D] copied
//      (the layouts attention wants), rotation on interleaved pairs (x[2i], x[2i+1]) by angle
//      t * theta^(-2i/D) from the fp32 cos/sin tables [T, D/2].
// bwd: dq, dk (rotated back by the inverse rotation), dv -> dqkv [B, T, (Hq + 2 Hkv) * D].
// One thread moves 8 elements (4 pairs): 16-B loads and stores; the thread index runs over
// (row, head, chunk) with the chunk fastest, so one head row of D = 128 is 256 contiguous bytes
// for 16 consecutive lanes on both sides. Replaces split + 2 transposes + fp32 round trip + stack
// + flatten per tensor on the torch path.
#include "vcx_common.h"

namespace vcx {

template <bool BWD>
__global__ void __launch_bounds__(256) rope_qkv_kernel(bf16* __restrict__ qkv, bf16* __restrict__ q,
                                                        bf16* __restrict__ k, bf16* __restrict__ v,
                                                        const float* __restrict__ cosv, const float* __restrict__ sinv,
                                                        int B, int T, int Hq, int Hkv, int D) {
  const int D8 = D >> 3, Htot = Hq + 2 * Hkv;
  const int64_t n = (int64_t)B * T * Htot * D8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(i % D8);
    const int64_t rest = i / D8;
    const int head = (int)(rest % Htot);
    const int64_t bt = rest / Htot;  // b * T + t
    const int t = (int)(bt % T), b = (int)(bt / T);
    bf16* tok = qkv + bt * (int64_t)Htot * D + (int64_t)head * D + c8 * 8;
    bf16* hm;  // the head-major tensor row [b, h, t, :]
    if (head < Hq)
      hm = q + (((int64_t)b * Hq + head) * T + t) * D;
    else if (head < Hq + Hkv)
      hm = k + (((int64_t)b * Hkv + head - Hq) * T + t) * D;
    else
      hm = v + (((int64_t)b * Hkv + head - Hq - Hkv) * T + t) * D;
    hm += c8 * 8;
    const bf16x8 x = BWD ? *(const bf16x8*)hm : *(const bf16x8*)tok;
    bf16x8 y;
    if (head < Hq + Hkv) {
      const f32x4 c = *(const f32x4*)(cosv + (int64_t)t * (D >> 1) + c8 * 4);
      const f32x4 s = *(const f32x4*)(sinv + (int64_t)t * (D >> 1) + c8 * 4);
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const float x0 = (float)x[2 * p], x1 = (float)x[2 * p + 1];
        if (BWD) {  // inverse rotation (transpose of the forward's)
          y[2 * p] = (bf16)fmaf(x0, c[p], x1 * s[p]);
          y[2 * p + 1] = (bf16)fmaf(x1, c[p], -x0 * s[p]);
        } else {
          y[2 * p] = (bf16)fmaf(x0, c[p], -x1 * s[p]);
          y[2 * p + 1] = (bf16)fmaf(x0, s[p], x1 * c[p]);
        }
      }
    } else {
      y = x;
    }
    if (BWD)
      *(bf16x8*)tok = y;
    else
      *(bf16x8*)hm = y;
  }
}

}  // namespace vcx

using namespace vcx;

void vcx_rope_qkv(void* qkv, void* q, void* k, void* v, const float* cosv, const float* sinv, int B, int T, int Hq,
                  int Hkv, int D, int backward, hipStream_t s) {
  const int64_t n = (int64_t)B * T * (Hq + 2 * Hkv) * (D / 8);
  const dim3 g(stream_grid(n, 256));
  if (backward)
    hipLaunchKernelGGL(rope_qkv_kernel<true>, g, dim3(256), 0, s, (bf16*)qkv, (bf16*)q, (bf16*)k, (bf16*)v, cosv, sinv,
                       B, T, Hq, Hkv, D);
  else
    hipLaunchKernelGGL(rope_qkv_kernel<false>, g, dim3(256), 0, s, (bf16*)qkv, (bf16*)q, (bf16*)k, (bf16*)v, cosv,
                       sinv, B, T, Hq, Hkv, D);
}
