// Train-mode BatchNorm fused with its ReLU and the residual add, channels-last (NHWC) bf16, for the
// ResNet-50 of BASELINE config 3 (models/resnet.py). Torch runs each of these as separate passes
// (batch statistics, normalise, add, ReLU; and in the backward ReLU', statistics of the gradient,
// input gradient), each reading or writing the whole activation; here:
//   forward : stats    (read x once: per-channel sum / sum of squares in fp32, block partials + atomics)
//             finalize (mean, 1/std, the per-channel affine scale/shift, running stats, num_batches_tracked)
//             apply    (read x [+ residual], write y = relu(x * scale + shift [+ residual]) and, with the
//                       ReLU, its mask as one BIT per element: 1 byte per lane of 8 channels)
//   backward: reduce   (read dy, mask, x: per-channel sum dz and sum dz * xhat, dz = dy * mask)
//             bwd_fin  (the sums for the dx pass; dbeta / dgamma added into the flat bf16 .grad when given)
//             dx       (read dy, mask, x, write dx [and d residual = dz])
// The bit mask replaces the bf16 y the backward passes used to read for [y > 0]: 1/16 of its bytes, so
// each backward pass moves ~2 B per element less (of ~8-10), and y need not be kept for the backward.
// The atomics accumulate into a zero-at-rest workspace (one per device, stream and C, owned by the
// binding) that the finalize kernels read and zero again: no fill kernel per call. (A last-block
// finalize inside the reduction kernels instead -- a ticket counter behind device-scope fences --
// measured 2x slower reductions, likely the device-scope fence in every block (on the 8-XCD chip it
// writes back / invalidates the XCD's L2; not profiled further): profiles/r4_resnet50_ab.txt.)
// Rows R = N * H * W, C channels (a power of two, 8 .. 2048); every lane moves 16 B (8 channels) per
// access. No reference analog (north-star config 3).
#include <cstdio>
#include <cstdlib>
#include <string>

#include "vcx_common.h"

namespace vcx {
namespace bn {

constexpr int NT = 256;
typedef float f32x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ void load8(const bf16* p, float (&v)[8]) {
  const bf16x8 x = *(const bf16x8*)p;
#pragma unroll
  for (int i = 0; i < 8; ++i) v[i] = (float)x[i];
}

template <int U>
struct Unroll {
  static constexpr int value = U;
};

// per-channel partial sums of this block over rows [r0, r1), reduced in LDS over the threads that
// share a channel chunk, then added to out0 / out1 (fp32 [C]) with one atomic per channel.
// body(off, step, Unroll<U>, s0, s1) handles the U rows off, off + step, ...: the main loop passes
// U = 4 so every lane keeps 4 row loads per operand in flight (one at a time left these passes at
// 2-3 TB/s, latency-bound: profiles/r5_cfg3_resnet50_categories.txt).
// channel_reduce_tail is the frame: main(r, step, rpp, ch, s0, s1) sums the full groups of rows from r and returns
// the first row it left; single rows finish with body(off, step, Unroll<1>, s0, s1); then the LDS reduction and
// the atomics
template <int BT, typename M, typename F>
__device__ __forceinline__ void channel_reduce_tail(int C, int64_t r0, int64_t r1, M&& main, F&& body, float* out0,
                                                    float* out1) {
  __shared__ float red[2][BT][9];  // [quantity][thread][8 channels + pad]
  const int tid = threadIdx.x;
  const int cpr = C / 8;                // chunks per row
  const int rpp = BT / cpr;             // rows per pass (>= 1)
  const int ch = tid % cpr, rr = tid / cpr;
  float s0[8], s1[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) s0[i] = s1[i] = 0.f;
  if (rr < rpp) {
    const int64_t step = (int64_t)rpp * C;
    int64_t r = main(r0 + rr, step, rpp, ch, s0, s1);
    for (; r < r1; r += rpp) body(r * C + ch * 8, step, Unroll<1>{}, s0, s1);
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    red[0][tid][i] = s0[i];
    red[1][tid][i] = s1[i];
  }
  __syncthreads();
  // thread t < C: channel t = chunk t / 8, element t % 8, summed over the rpp row slots
  for (int c = tid; c < C; c += BT) {
    const int k = c / 8, e = c % 8;
    float a = 0.f, b = 0.f;
    for (int q = 0; q < rpp; ++q) {
      a += red[0][k + q * cpr][e];
      b += red[1][k + q * cpr][e];
    }
    atomicAdd(out0 + c, a);
    atomicAdd(out1 + c, b);
  }
}

// groups of UR rows: issue UR rows, wait for all of them, sum, issue the next
template <int UR, int BT, typename F>
__device__ __forceinline__ void channel_reduce(int C, int64_t r0, int64_t r1, F&& body, float* out0, float* out1) {
  channel_reduce_tail<BT>(C, r0, r1, [&](int64_t r, int64_t step, int rpp, int ch, float(&s0)[8], float(&s1)[8]) {
    for (; r + (UR - 1) * rpp < r1; r += UR * rpp) body(r * C + ch * 8, step, Unroll<UR>{}, s0, s1);
    return r;
  }, body, out0, out1);
}

// pipelined (R = registers of U rows; ld(off, step, regs) / acc(regs, s0, s1) split body's load and sum): two
// register sets of U rows, the next set's loads issued before the current set is summed, so a lane's loads are
// never all retired at once. Measured (profiles/r6_bn_kernels.txt): the small late layers gain (bwd_reduce 398.1 ->
// 383.6 us per set of shapes), the 205 MB shapes stay at ~4.5 TB/s
template <int U, int BT, typename R, typename LD, typename ACC, typename F>
__device__ __forceinline__ void channel_reduce_pipe(int C, int64_t r0, int64_t r1, LD&& ld, ACC&& acc, F&& body,
                                                    float* out0, float* out1) {
  channel_reduce_tail<BT>(C, r0, r1, [&](int64_t r, int64_t step, int rpp, int ch, float(&s0)[8], float(&s1)[8]) {
    const int64_t span = (int64_t)U * rpp;
    R a, b;
    if (r + (U - 1) * rpp < r1) {
      ld(r * C + ch * 8, step, a);
      for (;;) {
        r += span;
        if (r + (U - 1) * rpp >= r1) {
          acc(a, s0, s1);
          break;
        }
        ld(r * C + ch * 8, step, b);
        acc(a, s0, s1);
        r += span;
        if (r + (U - 1) * rpp >= r1) {
          acc(b, s0, s1);
          break;
        }
        ld(r * C + ch * 8, step, a);
        acc(b, s0, s1);
      }
    }
    return r;
  }, body, out0, out1);
}

// sums of (x - k) and (x - k)^2 with a per-channel pivot k = x[row 0] (the same for every block):
// E[x^2] - m^2 on raw fp32 sums cancels catastrophically when |mean| >> std over millions of rows;
// shifted by a value of the batch, the sums are O(R std^2) and the variance keeps its digits
template <int U>
struct XRows {
  static constexpr int n = U;
  bf16x8 v[U];
};
template <int U>
struct DyXRows {
  static constexpr int n = U;
  bf16x8 g[U], x[U];
  unsigned mk[U];
};

// PIPE: channel_reduce_pipe with two sets of UR / 2 rows (the same rows in flight per lane)
template <int UR, int BT, bool PIPE = false>
__global__ void __launch_bounds__(BT) stats_kernel(const bf16* __restrict__ x, int64_t R, int C, int64_t rows_per_block,
                                                   float* __restrict__ sum, float* __restrict__ sumsq) {
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(R, r0 + rows_per_block);
  float k[8];
  load8(x + (threadIdx.x % (C / 8)) * 8, k);
  auto ld = [&](int64_t off, int64_t step, auto& g) {
#pragma unroll
    for (int j = 0; j < g.n; ++j) g.v[j] = *(const bf16x8*)(x + off + j * step);
  };
  auto acc = [&](const auto& g, float(&s0)[8], float(&s1)[8]) {
#pragma unroll
    for (int j = 0; j < g.n; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float d = (float)g.v[j][i] - k[i];
        s0[i] += d;
        s1[i] = fmaf(d, d, s1[i]);
      }
  };
  auto body = [&](int64_t off, int64_t step, auto u, float(&s0)[8], float(&s1)[8]) {
    XRows<decltype(u)::value> g;
    ld(off, step, g);
    acc(g, s0, s1);
  };
  if constexpr (PIPE)
    channel_reduce_pipe<UR / 2, BT, XRows<UR / 2>>(C, r0, r1, ld, acc, body, sum, sumsq);
  else
    channel_reduce<UR, BT>(C, r0, r1, body, sum, sumsq);
}

// mean, 1/std, scale = gamma/std, shift = beta - mean * scale; running stats (unbiased variance)
// updated in place in their own dtype (bf16 or fp32); num_batches_tracked + 1; ws = [sum | sumsq] of
// the pivot-shifted values (pivot = x[row 0], see stats_kernel), zeroed again for the next call
template <typename RT>
__global__ void finalize_kernel(float* __restrict__ ws, const bf16* __restrict__ x, int64_t R, int C,
                                const bf16* __restrict__ gamma,
                                const bf16* __restrict__ beta, float eps, float momentum, RT* __restrict__ run_mean,
                                RT* __restrict__ run_var, float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                float* __restrict__ scale, float* __restrict__ shift, int64_t* __restrict__ nbt) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c == 0 && nbt) *nbt += 1;
  if (c >= C) return;
  const float inv = 1.f / (float)R;
  const float d = ws[c] * inv;  // mean - pivot
  const float m = (float)x[c] + d;
  const float var = fmaxf(ws[C + c] * inv - d * d, 0.f);
  ws[c] = 0.f;
  ws[C + c] = 0.f;
  const float rs = rsqrtf(var + eps);
  const float g = (float)gamma[c], b = (float)beta[c];
  mean_out[c] = m;
  rstd_out[c] = rs;
  scale[c] = g * rs;
  shift[c] = b - m * g * rs;
  if (run_mean) {
    const float unb = R > 1 ? var * (float)R / (float)(R - 1) : var;
    run_mean[c] = (RT)((1.f - momentum) * (float)run_mean[c] + momentum * m);
    run_var[c] = (RT)((1.f - momentum) * (float)run_var[c] + momentum * unb);
  }
}

// the finalize of ONE channel from the raw pivot-shifted sums (see finalize_kernel)
struct ChanStats {
  float m, var, rs;
};
__device__ __forceinline__ ChanStats chan_stats(float s1, float s2, float pivot, float inv, float eps) {
  const float d = s1 * inv;
  const float var = fmaxf(s2 * inv - d * d, 0.f);
  return {pivot + d, var, rsqrtf(var + eps)};
}

// Per-layer workspace mode (FIN): the finalize runs inside the apply pass. Every thread derives the
// scale / shift of its 8 channels from the raw sums of the stats pass (ws[0, 2C)); block 0 also writes
// mean / 1/std / scale for the backward, the running stats and num_batches_tracked, and zeroes the
// layer's BACKWARD sums ws[2C, 4C) (their last reader, the previous step's dx pass, has finished; their
// next writer is this step's backward reduction). The forward sums are zeroed by the dx pass. One
// launch fewer per layer and direction (53 + 53 finalize launches of ~5 us in a ResNet-50 step).
struct FinArgs {
  float* ws;  // the layer's [fwd sum | fwd sumsq | bwd sum | bwd sumsq], fp32 [4C]
  const bf16 *gamma, *beta;
  void *run_mean, *run_var;
  int run_fp32;
  float eps, momentum, inv;
  int64_t R;
  float *mean, *rstd, *scale;
  int64_t* nbt;
};

// grid-stride loops whose stride (grid x 256 chunks) is a multiple of C / 8 (host check: C divides
// 2048): every thread keeps the same 8 channels, so their constants load once
template <bool RES, bool RELU, bool FIN>
__global__ void __launch_bounds__(NT) apply_kernel(const bf16* __restrict__ x, const bf16* __restrict__ res,
                                                   const float* __restrict__ scale, const float* __restrict__ shift,
                                                   bf16* __restrict__ y, unsigned char* __restrict__ mask, int64_t n8,
                                                   int cpr, FinArgs fa) {
  int64_t e = blockIdx.x * (int64_t)NT + threadIdx.x;
  const int c0 = (int)(e % cpr) * 8;
  float sc[8], sh[8];
  if constexpr (FIN) {
    // the block's channels' scale / shift once per block (a thread per channel) into LDS, read back by
    // every thread for its 8 channels (per-thread finalizes of all 8 channels made the pass 10-20 %
    // slower: dependent loads + rsqrt ahead of every thread's first row)
    __shared__ float s_sc[2048], s_sh[2048];
    const int C = cpr * 8;
    for (int c = threadIdx.x; c < C; c += NT) {
      const ChanStats st = chan_stats(fa.ws[c], fa.ws[C + c], (float)x[c], fa.inv, fa.eps);
      const float g = (float)fa.gamma[c] * st.rs;
      s_sc[c] = g;
      s_sh[c] = (float)fa.beta[c] - st.m * g;
      if (blockIdx.x == 0) {
        if (c == 0 && fa.nbt) *fa.nbt += 1;
        fa.mean[c] = st.m;
        fa.rstd[c] = st.rs;
        fa.scale[c] = g;
        fa.ws[2 * C + c] = 0.f;
        fa.ws[3 * C + c] = 0.f;
        if (fa.run_mean) {
          const float unb = fa.R > 1 ? st.var * (float)fa.R / (float)(fa.R - 1) : st.var, mo = fa.momentum;
          if (fa.run_fp32) {
            float* rm = (float*)fa.run_mean;
            float* rv = (float*)fa.run_var;
            rm[c] = (1.f - mo) * rm[c] + mo * st.m;
            rv[c] = (1.f - mo) * rv[c] + mo * unb;
          } else {
            bf16* rm = (bf16*)fa.run_mean;
            bf16* rv = (bf16*)fa.run_var;
            rm[c] = (bf16)((1.f - mo) * (float)rm[c] + mo * st.m);
            rv[c] = (bf16)((1.f - mo) * (float)rv[c] + mo * unb);
          }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = s_sc[c0 + i];
      sh[i] = s_sh[c0 + i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      sc[i] = scale[c0 + i];
      sh[i] = shift[c0 + i];
    }
  }
  for (; e < n8; e += (int64_t)gridDim.x * NT) {
    float v[8], r[8];
    load8(x + e * 8, v);
    if (RES) load8(res + e * 8, r);
    bf16x8 o;
    unsigned bits = 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      float z = fmaf(v[i], sc[i], sh[i]);
      if (RES) z += r[i];
      if (RELU) {
        bits |= (z > 0.f ? 1u : 0u) << i;
        z = fmaxf(z, 0.f);
      }
      o[i] = (bf16)z;
    }
    *(bf16x8*)(y + e * 8) = o;
    if (RELU && mask) mask[e] = (unsigned char)bits;
  }
}

// backward reductions: sum dz and sum dz * xhat per channel, dz = dy [* mask]
template <bool RELU, int UR, int BT, bool PIPE = false>
__global__ void __launch_bounds__(BT) bwd_reduce_kernel(const bf16* __restrict__ dy, const unsigned char* __restrict__ mask,
                                                        const bf16* __restrict__ x, const float* __restrict__ mean,
                                                        const float* __restrict__ rstd, int64_t R, int C,
                                                        int64_t rows_per_block, float* __restrict__ sdz,
                                                        float* __restrict__ sdzx) {
  const int64_t r0 = blockIdx.x * rows_per_block, r1 = min(R, r0 + rows_per_block);
  const int ch = (threadIdx.x % (C / 8)) * 8;
  float m[8], rs[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    m[i] = mean[ch + i];
    rs[i] = rstd[ch + i];
  }
  auto ld = [&](int64_t off, int64_t step, auto& g) {
#pragma unroll
    for (int j = 0; j < g.n; ++j) {
      g.g[j] = *(const bf16x8*)(dy + off + j * step);
      g.x[j] = *(const bf16x8*)(x + off + j * step);
      g.mk[j] = RELU ? mask[(off + j * step) >> 3] : 0xffu;
    }
  };
  auto acc = [&](const auto& g, float(&s0)[8], float(&s1)[8]) {
#pragma unroll
    for (int j = 0; j < g.n; ++j)
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float dz = RELU ? ((g.mk[j] >> i) & 1u ? (float)g.g[j][i] : 0.f) : (float)g.g[j][i];
        s0[i] += dz;
        s1[i] = fmaf(dz, ((float)g.x[j][i] - m[i]) * rs[i], s1[i]);
      }
  };
  auto body = [&](int64_t off, int64_t step, auto u, float(&s0)[8], float(&s1)[8]) {
    DyXRows<decltype(u)::value> g;
    ld(off, step, g);
    acc(g, s0, s1);
  };
  if constexpr (PIPE)
    channel_reduce_pipe<UR / 2, BT, DyXRows<UR / 2>>(C, r0, r1, ld, acc, body, sdz, sdzx);
  else
    channel_reduce<UR, BT>(C, r0, r1, body, sdz, sdzx);
}

// ws = [sum dz | sum dz xhat] -> sums (for the dx pass and the caller) and, when given, added into the
// flat bf16 gradients of beta / gamma; ws zeroed again for the next call
__global__ void bwd_finalize_kernel(float* __restrict__ ws, int C, float* __restrict__ sums, bf16* __restrict__ gw,
                                    bf16* __restrict__ gb) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float db = ws[c], dg = ws[C + c];
  ws[c] = 0.f;
  ws[C + c] = 0.f;
  sums[c] = db;
  sums[C + c] = dg;
  if (gb) gb[c] = (bf16)((float)gb[c] + db);
  if (gw) gw[c] = (bf16)((float)gw[c] + dg);
}

// dx = gamma rstd (dz - (sum dz + xhat sum dz xhat) / R); d residual = dz.
// FIN (per-layer workspace): sdz / sdzx are the layer's raw backward sums ws[2C, 4C) (no bwd_finalize
// launch); block 0 writes them to `sums`, adds dbeta / dgamma into gb / gw, and zeroes the layer's
// FORWARD sums ws[0, 2C) (last read by this step's apply pass; next written by the next forward)
template <bool RES, bool RELU, bool FIN>
__global__ void __launch_bounds__(NT) bwd_dx_kernel(const bf16* __restrict__ dy, const unsigned char* __restrict__ mask,
                                                    const bf16* __restrict__ x, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, const float* __restrict__ scale,
                                                    const float* __restrict__ sdz, const float* __restrict__ sdzx,
                                                    bf16* __restrict__ dx, bf16* __restrict__ dres, int64_t n8, int cpr,
                                                    float invR, float* __restrict__ fin_ws, float* __restrict__ sums,
                                                    bf16* __restrict__ gw, bf16* __restrict__ gb) {
  int64_t e = blockIdx.x * (int64_t)NT + threadIdx.x;
  const int c0 = (int)(e % cpr) * 8;
  if (FIN && blockIdx.x == 0) {
    const int C = cpr * 8;
    for (int c = threadIdx.x; c < C; c += NT) {
      const float db = sdz[c], dg = sdzx[c];
      sums[c] = db;
      sums[C + c] = dg;
      if (gb) gb[c] = (bf16)((float)gb[c] + db);
      if (gw) gw[c] = (bf16)((float)gw[c] + dg);
      fin_ws[c] = 0.f;
      fin_ws[C + c] = 0.f;
    }
  }
  float sc[8], m[8], rs[8], u[8], w[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    sc[i] = scale[c0 + i];
    m[i] = mean[c0 + i];
    rs[i] = rstd[c0 + i];
    u[i] = sdz[c0 + i] * invR;
    w[i] = sdzx[c0 + i] * invR;
  }
  for (; e < n8; e += (int64_t)gridDim.x * NT) {
    float g[8], xx[8];
    load8(dy + e * 8, g);
    load8(x + e * 8, xx);
    const unsigned mk = RELU ? mask[e] : 0xffu;
    bf16x8 o, od;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float dz = RELU ? ((mk >> i) & 1u ? g[i] : 0.f) : g[i];
      const float xh = (xx[i] - m[i]) * rs[i];
      o[i] = (bf16)(sc[i] * (dz - fmaf(xh, w[i], u[i])));
      od[i] = (bf16)dz;
    }
    *(bf16x8*)(dx + e * 8) = o;
    if (RES) *(bf16x8*)(dres + e * 8) = od;
  }
}

// ---- the ResNet stem's 3x3 / stride-2 / pad-1 max-pool on NHWC bf16, with a 1-byte window index per
// output element (kh * 3 + kw) instead of torch's int64 flat index, and a gather backward: each input
// element sums the gradients of the (at most 2 x 2) windows that picked it, so no zero fill + scatter.
// One thread per 8 channels of one output (forward) / input (backward) pixel.
typedef unsigned char u8x8 __attribute__((ext_vector_type(8)));

__global__ void __launch_bounds__(NT) maxpool_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                         unsigned char* __restrict__ idx, int N, int H, int W, int C,
                                                         int OH, int OW) {
  const int c8 = C / 8;
  const int64_t total = (int64_t)N * OH * OW * c8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cc = (int)(t % c8);
    int64_t r = t / c8;
    const int ow = (int)(r % OW);
    r /= OW;
    const int oh = (int)(r % OH);
    const int n = (int)(r / OH);
    float best[8];
    u8x8 arg;
    bool first = true;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * 2 - 1 + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = ow * 2 - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        float v[8];
        load8(x + (((int64_t)n * H + ih) * W + iw) * C + cc * 8, v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // the first in-window element, then strictly greater or NaN, and nothing replaces a NaN once
          // held (torch's order and NaN rule: `val > max || isnan(val)` against the running max)
          if (first || (best[e] == best[e] && !(v[e] <= best[e]))) {
            best[e] = v[e];
            arg[e] = (unsigned char)(kh * 3 + kw);
          }
        }
        first = false;
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)best[e];
    const int64_t off = (((int64_t)n * OH + oh) * OW + ow) * C + cc * 8;
    *(bf16x8*)(y + off) = o;
    *(u8x8*)(idx + off) = arg;
  }
}

__global__ void __launch_bounds__(NT) maxpool_bwd_kernel(const bf16* __restrict__ dy, const unsigned char* __restrict__ idx,
                                                         bf16* __restrict__ dx, int N, int H, int W, int C, int OH,
                                                         int OW) {
  const int c8 = C / 8;
  const int64_t total = (int64_t)N * H * W * c8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cc = (int)(t % c8);
    int64_t r = t / c8;
    const int iw = (int)(r % W);
    r /= W;
    const int ih = (int)(r % H);
    const int n = (int)(r / H);
    float acc[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[e] = 0.f;
    // windows oh with 2 oh - 1 <= ih <= 2 oh + 1
    const int oh0 = max(0, ih / 2), oh1 = min(OH - 1, (ih + 1) / 2);
    const int ow0 = max(0, iw / 2), ow1 = min(OW - 1, (iw + 1) / 2);
    for (int oh = oh0; oh <= oh1; ++oh) {
      const int kh = ih - (oh * 2 - 1);
      for (int ow = ow0; ow <= ow1; ++ow) {
        const int kw = iw - (ow * 2 - 1);
        const int64_t off = (((int64_t)n * OH + oh) * OW + ow) * C + cc * 8;
        const u8x8 a = *(const u8x8*)(idx + off);
        float g[8];
        load8(dy + off, g);
        const unsigned char k = (unsigned char)(kh * 3 + kw);
#pragma unroll
        for (int e = 0; e < 8; ++e)
          if (a[e] == k) acc[e] += g[e];
      }
    }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)acc[e];
    *(bf16x8*)(dx + (((int64_t)n * H + ih) * W + iw) * C + cc * 8) = o;
  }
}

// ---- ResNet strided-shortcut and pooling helpers on NHWC bf16 (C % 8 == 0), one lane per 8 channels of one
// pixel, 16-B accesses (torch's strided copy / add / broadcast for these ran at 1.4-2.3 TB/s in the config-3 step:
// scripts/cfg3_copy_sources.py)
// y[n, i, j] = x[n, i s, j s] (a stride-s 1x1 convolution's input)
__global__ void __launch_bounds__(NT) subsample_kernel(const bf16* __restrict__ x, bf16* __restrict__ y, int N, int H,
                                                       int W, int C, int s, int OH, int OW) {
  const int c8 = C / 8;
  const int64_t total = (int64_t)N * OH * OW * c8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cc = (int)(t % c8);
    const int64_t p = t / c8;  // output pixel
    const int j = (int)(p % OW);
    const int64_t q = p / OW;
    const int i = (int)(q % OH), n = (int)(q / OH);
    *(bf16x8*)(y + p * C + cc * 8) = *(const bf16x8*)(x + (((int64_t)n * H + i * s) * W + j * s) * C + cc * 8);
  }
}

// full[n, i s, j s] += g[n, i, j] (the stride-s shortcut's input gradient into the block input's)
__global__ void __launch_bounds__(NT) subsample_add_kernel(bf16* __restrict__ full, const bf16* __restrict__ g, int N,
                                                           int H, int W, int C, int s, int OH, int OW) {
  const int c8 = C / 8;
  const int64_t total = (int64_t)N * OH * OW * c8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cc = (int)(t % c8);
    const int64_t p = t / c8;
    const int j = (int)(p % OW);
    const int64_t q = p / OW;
    const int i = (int)(q % OH), n = (int)(q / OH);
    bf16* f = full + (((int64_t)n * H + i * s) * W + j * s) * C + cc * 8;
    const bf16x8 a = *(const bf16x8*)f, b = *(const bf16x8*)(g + p * C + cc * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)a[e] + (float)b[e]);
    *(bf16x8*)f = o;
  }
}

// out[n, h, w, c] = g[n, c] * scale (the global average pool's backward)
__global__ void __launch_bounds__(NT) bcast_hw_kernel(const bf16* __restrict__ g, bf16* __restrict__ out, int N, int HW,
                                                      int C, float scale) {
  const int c8 = C / 8;
  const int64_t total = (int64_t)N * HW * c8;
  for (int64_t t = blockIdx.x * (int64_t)NT + threadIdx.x; t < total; t += (int64_t)gridDim.x * NT) {
    const int cc = (int)(t % c8);
    const int n = (int)(t / ((int64_t)HW * c8));
    const bf16x8 v = *(const bf16x8*)(g + (int64_t)n * C + cc * 8);
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] = (bf16)((float)v[e] * scale);
    *(bf16x8*)(out + t * 8) = o;
  }
}

// reduction geometry (rows in flight per lane, target block count, minimum passes per block, threads per block).
// Round 6 default "w512p": w512q's geometry on channel_reduce_pipe (the next 4 rows' loads issued before the current
// 4 are summed): bwd_reduce 398.1 -> 383.6 us per set of shapes, the small late layers gaining, the 205 MB ones
// (dy and x together likely past the 256 MB last-level cache) at ~4.5 TB/s either way; config 3 ahead in 6 of 6
// interleaved pairs, +0.1..2.1 % (profiles/r6_bn_kernels.txt). "w512i" (the blocks sweeping the rows together,
// grid-stride, instead of a contiguous range each) measured 4-8 % slower on the large shapes: not kept.
// Before it, "w512q": 8 deep, ~256 blocks of 512 threads -- a quarter of the blocks, so a quarter of the
// per-block atomics into the layer's sums, which cost the statistics pass a third of its time at 1024 blocks
// (profiles/r6_bn_kernels.txt: stats 257.5 -> 200.0 us, reductions 420 -> 392 us per set of ResNet-50 shapes;
// config 3 9306 / 9318 vs 9222 / 9164 img/s, same box, interleaved). Round 5, config 3
// same box (gpurun_out/c16, c17): VCX_BN_REDUCE = "8n" (8 deep, ~1024 blocks of >= 32 passes;
// 8629-8722 img/s), "4" (4 deep, ~1024 blocks: 8556-8562), "8" (8 deep, ~2048 blocks of >= 16: 2 % under
// "4"), "4w" (4 deep, ~2048 blocks: 8380-8386) -- more blocks cost more than the small late layers gain
// (every block adds its partial sums into the workspace) -- and "8h" (8 deep, ~512 blocks)
struct ReduceGeo {
  int unroll, target, min_passes, threads = 256;
  bool pipe = false;  // channel_reduce_pipe
};
inline const ReduceGeo& reduce_geo() {
  static const ReduceGeo g = [] {
    const char* e = std::getenv("VCX_BN_REDUCE");
    const std::string v = e ? e : "w512p";
    if (v == "8") return ReduceGeo{8, 2048, 16};
    if (v == "4") return ReduceGeo{4, 1024, 32};
    if (v == "4w") return ReduceGeo{4, 2048, 16};
    if (v == "8h") return ReduceGeo{8, 512, 32};
    if (v == "w512") return ReduceGeo{8, 512, 32, 512};
    if (v == "8n") return ReduceGeo{8, 1024, 32};
    if (v == "w512q") return ReduceGeo{8, 256, 32, 512};
    if (v != "w512p") std::fprintf(stderr, "[vcx] VCX_BN_REDUCE=%s unknown, using w512p\n", v.c_str());
    return ReduceGeo{8, 256, 32, 512, true};
  }();
  return g;
}
inline int reduce_unroll() { return reduce_geo().unroll; }
inline int reduce_threads() { return reduce_geo().threads; }
inline bool reduce_pipe() { return reduce_geo().pipe; }
inline int64_t rows_per_block(int64_t R, int C) {
  const ReduceGeo& geo = reduce_geo();
  const int64_t rpp = geo.threads / (C / 8), target = geo.target, min_passes = geo.min_passes;
  int64_t rpb = (R + target - 1) / target;
  rpb = ((rpb + rpp - 1) / rpp) * rpp;
  return rpb < min_passes * rpp ? min_passes * rpp : rpb;
}
inline int grid_for(int64_t n8) {
  int64_t g = (n8 + NT - 1) / NT;
  return (int)(g < 8192 ? g : 8192);
}

}  // namespace bn
}  // namespace vcx

using namespace vcx;

// C a power of two in 8 .. 2048 (the grid-stride loops keep a thread on one channel chunk)
bool vcx_bn_supported(int C) { return C >= 8 && C <= 2048 && (2048 % C) == 0; }

// forward (train): ws = the zero-at-rest workspace, fp32 [2C] (zeroed once by the caller, left zeroed
// by every call); mean/rstd/scale/shift fp32 [C]; nbt int64 [1] or null.
// layer_ws: ws is instead the LAYER's own fp32 [4C] workspace (forward sums zero on entry, see
// apply_kernel FIN): no finalize launch, and the layer's backward sums are zeroed by the apply pass
void vcx_bn_fwd_train(const void* x, const void* res, void* y, void* mask, int64_t R, int C, const void* gamma,
                      const void* beta, void* run_mean, void* run_var, int run_fp32, float eps, float momentum, float* ws,
                      float* mean, float* rstd, float* scale, float* shift, int64_t* nbt, int relu, int layer_ws,
                      hipStream_t s) {
  using namespace bn;
  const int64_t rpb = rows_per_block(R, C);
  const int nb = (int)((R + rpb - 1) / rpb);
  if (reduce_pipe())
    hipLaunchKernelGGL((stats_kernel<8, 512, true>), dim3(nb), dim3(512), 0, s, (const bf16*)x, R, C, rpb, ws, ws + C);
  else if (reduce_threads() == 512)
    hipLaunchKernelGGL((stats_kernel<8, 512>), dim3(nb), dim3(512), 0, s, (const bf16*)x, R, C, rpb, ws, ws + C);
  else if (reduce_unroll() == 8)
    hipLaunchKernelGGL((stats_kernel<8, NT>), dim3(nb), dim3(NT), 0, s, (const bf16*)x, R, C, rpb, ws, ws + C);
  else
    hipLaunchKernelGGL((stats_kernel<4, NT>), dim3(nb), dim3(NT), 0, s, (const bf16*)x, R, C, rpb, ws, ws + C);
  FinArgs fa{ws, (const bf16*)gamma, (const bf16*)beta, run_mean, run_var, run_fp32, eps, momentum, 1.f / (float)R, R,
             mean, rstd, scale, nbt};
  if (!layer_ws) {
    if (run_fp32)
      hipLaunchKernelGGL(finalize_kernel<float>, dim3((C + 255) / 256), dim3(256), 0, s, ws, (const bf16*)x, R, C,
                         (const bf16*)gamma, (const bf16*)beta, eps, momentum, (float*)run_mean, (float*)run_var, mean,
                         rstd, scale, shift, nbt);
    else
      hipLaunchKernelGGL(finalize_kernel<bf16>, dim3((C + 255) / 256), dim3(256), 0, s, ws, (const bf16*)x, R, C,
                         (const bf16*)gamma, (const bf16*)beta, eps, momentum, (bf16*)run_mean, (bf16*)run_var, mean,
                         rstd, scale, shift, nbt);
  }
  const int64_t n8 = R * C / 8;
  const int g = layer_ws ? std::min(grid_for(n8), 2048) : grid_for(n8);  // FIN: a finalize per block
  auto go = [&](auto k) {
    hipLaunchKernelGGL(k, dim3(g), dim3(NT), 0, s, (const bf16*)x, (const bf16*)res, scale, shift, (bf16*)y,
                       (unsigned char*)mask, n8, C / 8, fa);
  };
  if (layer_ws) {
    if (res)
      relu ? go(apply_kernel<true, true, true>) : go(apply_kernel<true, false, true>);
    else
      relu ? go(apply_kernel<false, true, true>) : go(apply_kernel<false, false, true>);
  } else {
    if (res)
      relu ? go(apply_kernel<true, true, false>) : go(apply_kernel<true, false, false>);
    else
      relu ? go(apply_kernel<false, true, false>) : go(apply_kernel<false, false, false>);
  }
}

// y = act(x * scale + shift [+ res]) with given per-channel scale/shift (eval mode)
void vcx_bn_apply(const void* x, const void* res, void* y, int64_t R, int C, const float* scale, const float* shift,
                  int relu, hipStream_t s) {
  using namespace bn;
  const int64_t n8 = R * C / 8;
  const int g = grid_for(n8);
  const FinArgs fa{};
  auto go = [&](auto k) {
    hipLaunchKernelGGL(k, dim3(g), dim3(NT), 0, s, (const bf16*)x, (const bf16*)res, scale, shift, (bf16*)y,
                       (unsigned char*)nullptr, n8, C / 8, fa);
  };
  if (res)
    relu ? go(apply_kernel<true, true, false>) : go(apply_kernel<true, false, false>);
  else
    relu ? go(apply_kernel<false, true, false>) : go(apply_kernel<false, false, false>);
}

// backward: ws = the zero-at-rest workspace (as in the forward); sums = fp32 [2C] output [sum dz |
// sum dz xhat] = [dbeta | dgamma]; gw / gb = flat bf16 gradients of gamma / beta that dgamma / dbeta
// are added into (or null). layer_ws: ws is the layer's fp32 [4C] workspace (backward sums zero on
// entry): the reduction accumulates into ws[2C, 4C), the dx pass finalizes them and zeroes ws[0, 2C)
void vcx_bn_bwd(const void* dy, const void* mask, const void* x, const float* mean, const float* rstd, const float* scale,
                int64_t R, int C, float* ws, float* sums, void* gw, void* gb, void* dx, void* dres, int relu, int layer_ws,
                hipStream_t s) {
  using namespace bn;
  const int64_t rpb = rows_per_block(R, C);
  const int nb = (int)((R + rpb - 1) / rpb);
  float* bws = layer_ws ? ws + 2 * C : ws;
  const int bt = reduce_threads();
  auto red = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(nb), dim3(bt), 0, s, (const bf16*)dy, (const unsigned char*)mask, (const bf16*)x, mean,
                       rstd, R, C, rpb, bws, bws + C);
  };
  if (reduce_pipe())
    relu ? red(bwd_reduce_kernel<true, 8, 512, true>) : red(bwd_reduce_kernel<false, 8, 512, true>);
  else if (bt == 512)
    relu ? red(bwd_reduce_kernel<true, 8, 512>) : red(bwd_reduce_kernel<false, 8, 512>);
  else if (reduce_unroll() == 8)
    relu ? red(bwd_reduce_kernel<true, 8, NT>) : red(bwd_reduce_kernel<false, 8, NT>);
  else
    relu ? red(bwd_reduce_kernel<true, 4, NT>) : red(bwd_reduce_kernel<false, 4, NT>);
  if (!layer_ws)
    hipLaunchKernelGGL(bwd_finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, ws, C, sums, (bf16*)gw, (bf16*)gb);
  const float* sdz = layer_ws ? bws : sums;
  const int64_t n8 = R * C / 8;
  const int g = grid_for(n8);
  auto go = [&](auto k) {
    hipLaunchKernelGGL(k, dim3(g), dim3(NT), 0, s, (const bf16*)dy, (const unsigned char*)mask, (const bf16*)x, mean, rstd, scale,
                       sdz, sdz + C, (bf16*)dx, (bf16*)dres, n8, C / 8, 1.f / (float)R, ws, sums, (bf16*)gw, (bf16*)gb);
  };
  if (layer_ws) {
    if (dres)
      relu ? go(bwd_dx_kernel<true, true, true>) : go(bwd_dx_kernel<true, false, true>);
    else
      relu ? go(bwd_dx_kernel<false, true, true>) : go(bwd_dx_kernel<false, false, true>);
  } else {
    if (dres)
      relu ? go(bwd_dx_kernel<true, true, false>) : go(bwd_dx_kernel<true, false, false>);
    else
      relu ? go(bwd_dx_kernel<false, true, false>) : go(bwd_dx_kernel<false, false, false>);
  }
}

// y [N, OH, OW, C] = x[:, ::s, ::s, :]; full[:, ::s, ::s, :] += g; out [N, HW, C] = g [N, C] * scale (NHWC bf16)
void vcx_subsample_nhwc(const void* x, void* y, int N, int H, int W, int C, int s, hipStream_t st) {
  using namespace bn;
  const int OH = (H - 1) / s + 1, OW = (W - 1) / s + 1;
  hipLaunchKernelGGL(subsample_kernel, dim3(grid_for((int64_t)N * OH * OW * (C / 8))), dim3(NT), 0, st, (const bf16*)x,
                     (bf16*)y, N, H, W, C, s, OH, OW);
}

void vcx_subsample_add_nhwc(void* full, const void* g, int N, int H, int W, int C, int s, hipStream_t st) {
  using namespace bn;
  const int OH = (H - 1) / s + 1, OW = (W - 1) / s + 1;
  hipLaunchKernelGGL(subsample_add_kernel, dim3(grid_for((int64_t)N * OH * OW * (C / 8))), dim3(NT), 0, st, (bf16*)full,
                     (const bf16*)g, N, H, W, C, s, OH, OW);
}

void vcx_bcast_hw_nhwc(const void* g, void* out, int N, int HW, int C, float scale, hipStream_t st) {
  using namespace bn;
  hipLaunchKernelGGL(bcast_hw_kernel, dim3(grid_for((int64_t)N * HW * (C / 8))), dim3(NT), 0, st, (const bf16*)g,
                     (bf16*)out, N, HW, C, scale);
}

// stem max-pool 3x3 / stride 2 / pad 1, NHWC bf16 (C % 8 == 0): y, idx [N, OH, OW, C]
void vcx_maxpool3s2_fwd(const void* x, void* y, void* idx, int N, int H, int W, int C, int OH, int OW, hipStream_t s) {
  using namespace bn;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for(total)), dim3(NT), 0, s, (const bf16*)x, (bf16*)y,
                     (unsigned char*)idx, N, H, W, C, OH, OW);
}

void vcx_maxpool3s2_bwd(const void* dy, const void* idx, void* dx, int N, int H, int W, int C, int OH, int OW,
                        hipStream_t s) {
  using namespace bn;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for(total)), dim3(NT), 0, s, (const bf16*)dy,
                     (const unsigned char*)idx, (bf16*)dx, N, H, W, C, OH, OW);
}
