// LayerNorm (+ fused residual add), RMSNorm, tanh-GELU and fused softmax-cross-entropy
// kernels for the transformer training path (gfx950).
//
// Shape rules (checked host-side in the binding): row length C % 8 == 0, C <= 8192.
// One wave64 owns one row; a 256-thread block covers 4 rows. The row is held in registers
// (CH = ceil(C/512) chunks of 8 elements per lane), so the variance is an exact two-pass
// computation over registers with a single HBM read of the row.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "vcx_api.h"
#include "vcx_common.h"

namespace vcx {

// ============================================================ LayerNorm forward
// xsum = a + b [+ bb] (if b != nullptr, written to xout), y = LN(xsum) * w + bias
// bb is the bias of the GEMM that produced b (its epilogue add is moved here for free; the
// matching bias gradient falls out of the backward's column sums)
template <int CH>
__global__ void __launch_bounds__(256) ln_fwd_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                      bf16* __restrict__ xout, bf16* __restrict__ y,
                                                      const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      int R, int C, float eps, int rms, const bf16* __restrict__ bb) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= R) return;
  const int C8 = C >> 3;
  const int64_t off = (int64_t)row * C;
  float v[CH][8];
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = lane + k * 64;
    if (c < C8) {
      bf16x8 av = *(const bf16x8*)(a + off + c * 8);
      if (b) {
        bf16x8 bv = *(const bf16x8*)(b + off + c * 8);
        bf16x8 s;
        float bias_b[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (bb) {
          bf16x8 t = *(const bf16x8*)(bb + c * 8);
#pragma unroll
          for (int j = 0; j < 8; ++j) bias_b[j] = (float)t[j];
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          s[j] = (bf16)((float)av[j] + ((float)bv[j] + bias_b[j]));
          v[k][j] = (float)s[j];  // normalise the rounded residual actually stored
        }
        *(bf16x8*)(xout + off + c * 8) = s;
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) v[k][j] = (float)av[j];
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sum += v[k][j];
    }
  }
  const float invC = 1.f / (float)C;
  float mean = rms ? 0.f : wave_sum(sum) * invC;
  float var = 0.f;
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = lane + k * 64;
    if (c < C8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float d = v[k][j] - mean;
        var = fmaf(d, d, var);
      }
    }
  }
  var = wave_sum(var) * invC;
  const float rstd = rsqrtf(var + eps);
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = lane + k * 64;
    if (c < C8) {
      bf16x8 wv = *(const bf16x8*)(w + c * 8);
      bf16x8 o;
      if (bias) {
        bf16x8 bv = *(const bf16x8*)(bias + c * 8);
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)fmaf((v[k][j] - mean) * rstd, (float)wv[j], (float)bv[j]);
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) o[j] = (bf16)((v[k][j] - mean) * rstd * (float)wv[j]);
      }
      *(bf16x8*)(y + off + c * 8) = o;
    }
  }
  if (lane == 0) {
    mean_out[row] = mean;
    rstd_out[row] = rstd;
  }
}

// Row lengths that are a multiple of 256 (GPT-2: C = 768): every lane holds Q chunks of 4
// elements (8-B accesses, all 64 lanes busy; the 8-element form leaves half the lanes idle in
// the last chunk at C = 768), and each wave walks rows gw, gw + nw, ... with the next row's a/b
// loads issued before this row's two cross-lane reductions (a one-row software pipeline, as in
// the backward), so every lane keeps 2 x Q loads in flight through the shuffles.
template <int Q>
__global__ void __launch_bounds__(256) ln_fwd4_kernel(const bf16* __restrict__ a, const bf16* __restrict__ b,
                                                       bf16* __restrict__ xout, bf16* __restrict__ y,
                                                       const bf16* __restrict__ w, const bf16* __restrict__ bias,
                                                       float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                       int R, int C, float eps, int rms, const bf16* __restrict__ bb) {
  const int lane = threadIdx.x & 63;
  const int nw = gridDim.x * 4, gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  float wv[Q][4], bv_[Q][4], bbv[Q][4];
#pragma unroll
  for (int k = 0; k < Q; ++k) {
    const int c = k * 256 + lane * 4;
    const bf16x4 t = *(const bf16x4*)(w + c);
    const bf16x4 u = bias ? *(const bf16x4*)(bias + c) : bf16x4{};
    const bf16x4 v = bb ? *(const bf16x4*)(bb + c) : bf16x4{};
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      wv[k][j] = (float)t[j];
      bv_[k][j] = bias ? (float)u[j] : 0.f;
      bbv[k][j] = bb ? (float)v[j] : 0.f;
    }
  }
  const float invC = 1.f / (float)C;
  bf16x4 av[Q], bvv[Q];
  auto load_row = [&](int row, bf16x4(&aa)[Q], bf16x4(&bbx)[Q]) {
    const int64_t off = (int64_t)row * C + lane * 4;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      aa[k] = *(const bf16x4*)(a + off + k * 256);
      if (b) bbx[k] = *(const bf16x4*)(b + off + k * 256);
    }
  };
  if (gw < R) load_row(gw, av, bvv);
  for (int row = gw; row < R; row += nw) {
    bf16x4 nav[Q], nbv[Q];
    const int nxt = row + nw;
    if (nxt < R) load_row(nxt, nav, nbv);
    const int64_t off = (int64_t)row * C + lane * 4;
    float v[Q][4];
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      if (b) {
        bf16x4 sres;
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          sres[j] = (bf16)((float)av[k][j] + ((float)bvv[k][j] + bbv[k][j]));
          v[k][j] = (float)sres[j];  // normalise the rounded residual actually stored
        }
        *(bf16x4*)(xout + off + k * 256) = sres;
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[k][j] = (float)av[k][j];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) sum += v[k][j];
    }
    const float mean = rms ? 0.f : wave_sum(sum) * invC;
    float var = 0.f;
#pragma unroll
    for (int k = 0; k < Q; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float d = v[k][j] - mean;
        var = fmaf(d, d, var);
      }
    const float rstd = rsqrtf(wave_sum(var) * invC + eps);
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      bf16x4 o;
#pragma unroll
      for (int j = 0; j < 4; ++j) o[j] = (bf16)fmaf((v[k][j] - mean) * rstd, wv[k][j], bv_[k][j]);
      *(bf16x4*)(y + off + k * 256) = o;
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
#pragma unroll
    for (int k = 0; k < Q; ++k) {
      av[k] = nav[k];
      if (b) bvv[k] = nbv[k];
    }
  }
}

// ============================================================ LayerNorm backward
// dx = rstd * (w*dy - mean(w*dy) - xhat * mean(w*dy*xhat)) + dres
// per-wave partial dw = sum_rows dy*xhat, db = sum_rows dy -> part[(wave_global), C]
// Each wave walks rows gw, gw + nw, ... with a one-row software pipeline: the next row's dy, x,
// dres, mean and rstd loads are issued before this row's two cross-lane reductions, so every
// lane keeps (2 or 3) x CH 16-B loads in flight through the shuffles (the row loop is otherwise
// latency-bound at ~3.5 TB/s). RES is a template flag so no load sits behind a runtime branch.
// VEC = elements per lane access: 8 (16-B loads) in general; 4 (8-B loads) when the row is a
// multiple of 256 but not of 512 elements (C = 768: 3 chunks on every lane instead of 2 on half
// the lanes and 1 on the rest; 140 instead of 182 VGPRs: 3 instead of 2 waves per SIMD, so 1.5x the
// bytes in flight per CU). Forcing 4 waves per SIMD spills.
template <int CH, bool RES, int VEC>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(VEC == 4 ? 3 : 1))) ln_bwd_kernel(const bf16* __restrict__ dy, const bf16* __restrict__ x,
                                                      const bf16* __restrict__ w, const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in,
                                                      const bf16* __restrict__ dres, bf16* __restrict__ dx,
                                                      float* __restrict__ dw_part, float* __restrict__ db_part,
                                                      int R, int C, int rms, float* __restrict__ dbb_part) {
  const int lane = threadIdx.x & 63;
  const int gw = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nw = gridDim.x * 4;
  using BV = std::conditional_t<VEC == 8, bf16x8, bf16x4>;
  const int C8 = C / VEC;  // VEC-element chunks per row
  const float invC = 1.f / (float)C;
  float dwacc[CH][VEC], dbacc[CH][VEC], wreg[CH][VEC], dxacc[CH][VEC];
#pragma unroll
  for (int k = 0; k < CH; ++k) {
    const int c = lane + k * 64;
#pragma unroll
    for (int j = 0; j < VEC; ++j) {
      dwacc[k][j] = 0.f;
      dbacc[k][j] = 0.f;
      wreg[k][j] = 0.f;
      dxacc[k][j] = 0.f;
    }
    if (c < C8) {
      BV wv = *(const BV*)(w + c * VEC);
#pragma unroll
      for (int j = 0; j < VEC; ++j) wreg[k][j] = (float)wv[j];
    }
  }
  BV cd[CH], cx[CH], cr[CH];
  float cmean = 0.f, crstd = 0.f;
  auto load = [&](int row, BV(&d)[CH], BV(&xv)[CH], BV(&rv)[CH], float& mu, float& rs) {
    const int64_t off = (int64_t)row * C;
    mu = mean_in[row];
    rs = rstd_in[row];
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int c = lane + k * 64;
      if (c < C8) {
        d[k] = *(const BV*)(dy + off + c * VEC);
        xv[k] = *(const BV*)(x + off + c * VEC);
        if (RES) rv[k] = *(const BV*)(dres + off + c * VEC);
      }
    }
  };
  if (gw < R) load(gw, cd, cx, cr, cmean, crstd);
  for (int row = gw; row < R; row += nw) {
    BV nd[CH], nx[CH], nr[CH];
    float nmean = 0.f, nrstd = 0.f;
    if (row + nw < R) load(row + nw, nd, nx, nr, nmean, nrstd);
    const int64_t off = (int64_t)row * C;
    float s1 = 0.f, s2 = 0.f;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int c = lane + k * 64;
      if (c < C8) {
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float d = (float)cd[k][j];
          const float xh = ((float)cx[k][j] - cmean) * crstd;
          const float g = d * wreg[k][j];
          s1 += g;
          s2 = fmaf(g, xh, s2);
          dwacc[k][j] = fmaf(d, xh, dwacc[k][j]);
          dbacc[k][j] += d;
        }
      }
    }
    s1 = rms ? 0.f : wave_sum(s1) * invC;
    s2 = wave_sum(s2) * invC;
    // dx = rstd*(g - s1) - xhat*rstd*s2 with g and xhat recomputed from the loaded bf16 row (written
    // as different expressions so they are not merged with the first pass's values and kept alive:
    // 2 x CH x VEC fewer live registers through the reductions)
    const float k2 = crstd * crstd * s2, mk2 = cmean * k2;
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int c = lane + k * 64;
      if (c < C8) {
        BV o;
#pragma unroll
        for (int j = 0; j < VEC; ++j) {
          const float gs = fmaf((float)cd[k][j], wreg[k][j], -s1);
          const float v = fmaf(crstd, gs, -fmaf((float)cx[k][j], k2, -mk2)) + (RES ? (float)cr[k][j] : 0.f);
          o[j] = (bf16)v;
          dxacc[k][j] += v;
        }
        *(BV*)(dx + off + c * VEC) = o;
      }
    }
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      cd[k] = nd[k];
      cx[k] = nx[k];
      if (RES) cr[k] = nr[k];
    }
    cmean = nmean;
    crstd = nrstd;
  }
  if constexpr (CH * VEC <= 32) {
    // sum the 4 waves' column partials in LDS: ONE partial row per block (4x less partial traffic
    // for the column-sum kernels: 9 instead of 38 MB per call at the GPT-2 bench shape)
    __shared__ __attribute__((aligned(16))) float red[4][CH * 64 * VEC];
    const int w = threadIdx.x >> 6;
    auto reduce_out = [&](float(&acc)[CH][VEC], float* part) {
#pragma unroll
      for (int k = 0; k < CH; ++k) {
        const int c = lane + k * 64;
        if (c < C8) {
#pragma unroll
          for (int j = 0; j < VEC; j += 4)
            *(f32x4*)(&red[w][c * VEC + j]) = f32x4{acc[k][j], acc[k][j + 1], acc[k][j + 2], acc[k][j + 3]};
        }
      }
      __syncthreads();
      for (int i = threadIdx.x; i < C; i += 256)
        part[(int64_t)blockIdx.x * C + i] = (red[0][i] + red[1][i]) + (red[2][i] + red[3][i]);
      __syncthreads();
    };
    reduce_out(dwacc, dw_part);
    if (db_part) reduce_out(dbacc, db_part);
    if (dbb_part) reduce_out(dxacc, dbb_part);  // gradient of the branch bias = column sums of dx
  } else {
    static_assert(VEC == 8, "per-wave partial rows are written as 8-column chunks");
#pragma unroll
    for (int k = 0; k < CH; ++k) {
      const int c = lane + k * 64;
      if (c < C8) {
        float* dwp = dw_part + (int64_t)gw * C + c * 8;
        *(f32x4*)dwp = f32x4{dwacc[k][0], dwacc[k][1], dwacc[k][2], dwacc[k][3]};
        *(f32x4*)(dwp + 4) = f32x4{dwacc[k][4], dwacc[k][5], dwacc[k][6], dwacc[k][7]};
        if (db_part) {
          float* dbp = db_part + (int64_t)gw * C + c * 8;
          *(f32x4*)dbp = f32x4{dbacc[k][0], dbacc[k][1], dbacc[k][2], dbacc[k][3]};
          *(f32x4*)(dbp + 4) = f32x4{dbacc[k][4], dbacc[k][5], dbacc[k][6], dbacc[k][7]};
        }
        if (dbb_part) {  // gradient of the branch bias = column sums of dx
          float* p = dbb_part + (int64_t)gw * C + c * 8;
          *(f32x4*)p = f32x4{dxacc[k][0], dxacc[k][1], dxacc[k][2], dxacc[k][3]};
          *(f32x4*)(p + 4) = f32x4{dxacc[k][4], dxacc[k][5], dxacc[k][6], dxacc[k][7]};
        }
      }
    }
  }
}

// ============================================================ bias + tanh-GELU over [R, F]
// fwd: y = gelu(x + b). bwd: dx = dy * gelu'(x + b) and per-block column partials of dx
// (the bias gradient) — the GEMM before it runs without a bias epilogue and no separate
// bias-gradient reduction is needed. grid = (ceil(F/8/256), row groups).
__device__ __forceinline__ float gelu_f(float x);
__device__ __forceinline__ float gelu_grad_f(float x);

// bias + GELU over [R, F] row-major: a block is TPB threads x 8 columns; each thread walks rows
// r = blockIdx.y + k * gridDim.y with 4 rows' loads in flight (16-B vectors)
template <int TPB>
__global__ void __launch_bounds__(TPB) bias_gelu_fwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ b,
                                                            bf16* __restrict__ y, int R, int F) {
  const int c8 = blockIdx.x * TPB + threadIdx.x;
  if (c8 * 8 >= F) return;
  bf16x8 bv = *(const bf16x8*)(b + c8 * 8);
  float bf[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) bf[j] = (float)bv[j];
  const int G = gridDim.y;
  int r = blockIdx.y;
  // 4 rows per step, software-pipelined like the backward: the next step's loads are in flight
  // during this step's math and stores
  bf16x8 v[4];
  auto load4 = [&](int r0, bf16x8(&vv)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) vv[u] = *(const bf16x8*)(x + (int64_t)(r0 + u * G) * F + c8 * 8);
  };
  if (r + 3 * G < R) load4(r, v);
  for (; r + 3 * G < R; r += 4 * G) {
    bf16x8 nv[4];
    const bool more = r + 7 * G < R;
    if (more) load4(r + 4 * G, nv);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_f((float)v[u][j] + bf[j]);
      *(bf16x8*)(y + (int64_t)(r + u * G) * F + c8 * 8) = o;
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < 4; ++u) v[u] = nv[u];
    }
  }
  for (; r < R; r += G) {
    const int64_t off = (int64_t)r * F + c8 * 8;
    bf16x8 v1 = *(const bf16x8*)(x + off);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_f((float)v1[j] + bf[j]);
    *(bf16x8*)(y + off) = o;
  }
}

template <int TPB>
__global__ void __launch_bounds__(TPB) bias_gelu_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ b,
                                                            const bf16* __restrict__ dy, bf16* __restrict__ dx,
                                                            float* __restrict__ dbias_part, int R, int F) {
  const int c8 = blockIdx.x * TPB + threadIdx.x;
  if (c8 * 8 >= F) return;
  bf16x8 bv = *(const bf16x8*)(b + c8 * 8);
  float bf[8], acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    bf[j] = (float)bv[j];
    acc[j] = 0.f;
  }
  const int G = gridDim.y;
  int r = blockIdx.y;
  // 4 rows per step, software-pipelined: the next step's 8 loads are issued before this step's
  // math and stores, so each lane keeps 16 loads in flight across the step boundary
  bf16x8 v[4], g[4];
  auto load4 = [&](int r0, bf16x8(&vv)[4], bf16x8(&gg)[4]) {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int64_t off = (int64_t)(r0 + u * G) * F + c8 * 8;
      vv[u] = *(const bf16x8*)(x + off);
      gg[u] = *(const bf16x8*)(dy + off);
    }
  };
  if (r + 3 * G < R) load4(r, v, g);
  for (; r + 3 * G < R; r += 4 * G) {
    bf16x8 nv[4], ng[4];
    const bool more = r + 7 * G < R;
    if (more) load4(r + 4 * G, nv, ng);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float d = (float)g[u][j] * gelu_grad_f((float)v[u][j] + bf[j]);
        o[j] = (bf16)d;
        acc[j] += d;
      }
      *(bf16x8*)(dx + (int64_t)(r + u * G) * F + c8 * 8) = o;
    }
    if (more) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        v[u] = nv[u];
        g[u] = ng[u];
      }
    }
  }
  for (; r < R; r += G) {
    const int64_t off = (int64_t)r * F + c8 * 8;
    bf16x8 v1 = *(const bf16x8*)(x + off);
    bf16x8 g1 = *(const bf16x8*)(dy + off);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = (float)g1[j] * gelu_grad_f((float)v1[j] + bf[j]);
      o[j] = (bf16)d;
      acc[j] += d;
    }
    *(bf16x8*)(dx + off) = o;
  }
  float* p = dbias_part + (int64_t)blockIdx.y * F + c8 * 8;
  *(f32x4*)p = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *(f32x4*)(p + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}



// Column partial sums of a bf16 [R, F] matrix (the bias gradient of a token-major GEMM output):
// same geometry as bias_gelu_bwd without the GELU, 4 rows' 16-B loads in flight per thread.
template <int TPB>
__global__ void __launch_bounds__(TPB) colsum_part_bf16_kernel(const bf16* __restrict__ y, float* __restrict__ part,
                                                               int R, int F) {
  const int c8 = blockIdx.x * TPB + threadIdx.x;
  if (c8 * 8 >= F) return;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  const int G = gridDim.y;
  int r = blockIdx.y;
  for (; r + 3 * G < R; r += 4 * G) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *(const bf16x8*)(y + (int64_t)(r + u * G) * F + c8 * 8);
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += (float)v[u][j];
  }
  for (; r < R; r += G) {
    bf16x8 v = *(const bf16x8*)(y + (int64_t)r * F + c8 * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += (float)v[j];
  }
  float* p = part + (int64_t)blockIdx.y * F + c8 * 8;
  *(f32x4*)p = f32x4{acc[0], acc[1], acc[2], acc[3]};
  *(f32x4*)(p + 4) = f32x4{acc[4], acc[5], acc[6], acc[7]};
}

// Two-stage column sums of up to three [P, C] fp32 partial buffers -> bf16 [C] each, in two
// launches for all outputs together. Stage 1: grid (C/64, NB, nout) -- every block reduces
// P/NB rows of 64 columns (4 waves, LDS combine) into stage[out][NB][C]; stage 2: NB rows -> bf16.
// (A single-stage sum had only C/64 blocks -- 12 for C = 768 -- and ran latency-bound.)
__global__ void __launch_bounds__(256) colsum_stage1_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                            const float* __restrict__ p2, float* __restrict__ stage,
                                                            int P, int C) {
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int out = blockIdx.z, NB = gridDim.y, by = blockIdx.y;
  const float* part = out == 0 ? p0 : (out == 1 ? p1 : p2);
  const int c = blockIdx.x * 64 + lane;
  const int r0 = (int)((int64_t)P * by / NB), r1 = (int)((int64_t)P * (by + 1) / NB);
  float acc = 0.f;
  if (c < C) {
    int r = r0 + w;
    for (; r + 12 < r1; r += 16) {
      const float a0 = part[(int64_t)r * C + c], a1 = part[(int64_t)(r + 4) * C + c];
      const float a2 = part[(int64_t)(r + 8) * C + c], a3 = part[(int64_t)(r + 12) * C + c];
      acc += (a0 + a1) + (a2 + a3);
    }
    for (; r < r1; r += 4) acc += part[(int64_t)r * C + c];
  }
  red[w][lane] = acc;
  __syncthreads();
  if (w == 0 && c < C) stage[((int64_t)out * NB + by) * C + c] = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
}

__global__ void __launch_bounds__(64) colsum_stage2_kernel(const float* __restrict__ stage, int NB, int C,
                                                           bf16* __restrict__ o0, bf16* __restrict__ o1,
                                                           bf16* __restrict__ o2, int accum_mask) {
  const int out = blockIdx.y;
  const int c = blockIdx.x * 64 + threadIdx.x;
  if (c >= C) return;
  const float* st = stage + (int64_t)out * NB * C + c;
  // NB is always VCX_COLSUM_NB: fully unrolled so all loads are in flight at once instead of a
  // chain of dependent L2 round trips
  float v[VCX_COLSUM_NB];
#pragma unroll
  for (int i = 0; i < VCX_COLSUM_NB; ++i) v[i] = st[(int64_t)i * C];
  float acc = 0.f;
#pragma unroll
  for (int i = 0; i < VCX_COLSUM_NB; ++i) acc += v[i];
  bf16* o = out == 0 ? o0 : (out == 1 ? o1 : o2);
  if ((accum_mask >> out) & 1) acc += (float)o[c];  // add into an existing (flat) gradient
  o[c] = (bf16)acc;
}

// ============================================================ tanh-GELU
// 0.5 x (1 + tanh(u)) == x * sigmoid(2u): one exp2 and one reciprocal instead of a libm tanhf
__device__ __forceinline__ float gelu_f(float x) {
  const float c0 = -2.f * 0.7978845608028654f * 1.4426950408889634f, k1 = 0.044715f;
  const float e = __builtin_amdgcn_exp2f(c0 * fmaf(k1 * x, x * x, x));  // exp(-2u)
  return x * __builtin_amdgcn_rcpf(1.f + e);
}
__device__ __forceinline__ float gelu_grad_f(float x) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float c0 = -2.f * k0 * 1.4426950408889634f;
  const float x2 = x * x;
  const float e = __builtin_amdgcn_exp2f(c0 * fmaf(k1 * x, x2, x));
  const float sg = __builtin_amdgcn_rcpf(1.f + e);  // sigmoid(2u)
  const float du2 = 2.f * k0 * fmaf(3.f * k1, x2, 1.f);
  return fmaf(x * sg * (1.f - sg), du2, sg);
}

__global__ void __launch_bounds__(256) gelu_fwd_kernel(const bf16* __restrict__ x, bf16* __restrict__ y,
                                                        int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    bf16x8 v = *(const bf16x8*)(x + i * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)gelu_f((float)v[j]);
    *(bf16x8*)(y + i * 8) = o;
  }
}

__global__ void __launch_bounds__(256) gelu_bwd_kernel(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        bf16* __restrict__ dx, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    bf16x8 v = *(const bf16x8*)(x + i * 8);
    bf16x8 g = *(const bf16x8*)(dy + i * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)g[j] * gelu_grad_f((float)v[j]));
    *(bf16x8*)(dx + i * 8) = o;
  }
}

// SwiGLU for the Llama MLP: y = silu(g) * u, over [R, 2F] packed as [g | u] per row.
__global__ void __launch_bounds__(256) swiglu_fwd_kernel(const bf16* __restrict__ gu, bf16* __restrict__ y,
                                                          int64_t R, int F) {
  const int F8 = F >> 3;
  const int64_t n8 = R * F8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / F8, c = i - r * F8;
    bf16x8 g = *(const bf16x8*)(gu + r * 2 * F + c * 8);
    bf16x8 u = *(const bf16x8*)(gu + r * 2 * F + F + c * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gf = (float)g[j];
      o[j] = (bf16)(gf / (1.f + __expf(-gf)) * (float)u[j]);
    }
    *(bf16x8*)(y + r * F + c * 8) = o;
  }
}

__global__ void __launch_bounds__(256) swiglu_bwd_kernel(const bf16* __restrict__ gu, const bf16* __restrict__ dy,
                                                          bf16* __restrict__ dgu, int64_t R, int F) {
  const int F8 = F >> 3;
  const int64_t n8 = R * F8;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / F8, c = i - r * F8;
    bf16x8 g = *(const bf16x8*)(gu + r * 2 * F + c * 8);
    bf16x8 u = *(const bf16x8*)(gu + r * 2 * F + F + c * 8);
    bf16x8 d = *(const bf16x8*)(dy + r * F + c * 8);
    bf16x8 dg, du;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float gf = (float)g[j], uf = (float)u[j], df = (float)d[j];
      float sg = 1.f / (1.f + __expf(-gf));
      float silu = gf * sg;
      du[j] = (bf16)(df * silu);
      dg[j] = (bf16)(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    *(bf16x8*)(dgu + r * 2 * F + c * 8) = dg;
    *(bf16x8*)(dgu + r * 2 * F + F + c * 8) = du;
  }
}

// ============================================================ cross-entropy
// logits [R, Vp] bf16 (Vp = padded row stride, only the first V columns are real classes).
// fwd: lse[r], loss[r] = lse - logit[target] (0 for target < 0 = ignore)
__global__ void __launch_bounds__(256) xent_fwd_kernel(const bf16* __restrict__ logits, const int64_t* __restrict__ tgt,
                                                        float* __restrict__ lse_out, float* __restrict__ loss_out,
                                                        int V, int Vp) {
  __shared__ float sm[4], ss[4];
  const int64_t row = blockIdx.x;
  const bf16* lr = logits + row * Vp;
  const int V8 = V >> 3;  // full chunks
  float m = -INFINITY, s = 0.f;
  for (int c = threadIdx.x; c < V8; c += 256) {
    bf16x8 v = *(const bf16x8*)(lr + c * 8);
    float f[8], cm = -INFINITY;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      f[j] = (float)v[j];
      cm = fmaxf(cm, f[j]);
    }
    if (cm > m) {
      s *= __expf(m - cm);
      m = cm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) s += __expf(f[j] - m);
  }
  for (int c = V8 * 8 + threadIdx.x; c < V; c += 256) {  // ragged tail (V % 8)
    float f = (float)lr[c];
    if (f > m) {
      s *= __expf(m - f);
      m = f;
    }
    s += __expf(f - m);
  }
  // wave merge of (m, s)
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    float om = __shfl_xor(m, o, 64), os = __shfl_xor(s, o, 64);
    float nm = fmaxf(m, om);
    s = (m == -INFINITY ? 0.f : s * __expf(m - nm)) + (om == -INFINITY ? 0.f : os * __expf(om - nm));
    m = nm;
  }
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) {
    sm[wid] = m;
    ss[wid] = s;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float M = sm[0];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[i]);
    float S = 0.f;
    for (int i = 0; i < 4; ++i) S += (sm[i] == -INFINITY) ? 0.f : ss[i] * __expf(sm[i] - M);
    const float lse = M + __logf(S);
    lse_out[row] = lse;
    const int64_t t = tgt[row];
    loss_out[row] = (t >= 0 && t < V) ? (lse - (float)lr[t]) : 0.f;
  }
}

// bwd (in place allowed: dlogits may alias logits):
//   d[r, c] = gscale * (exp(logit - lse) - [c == target])  for c < V,  0 for V <= c < Vp
__global__ void __launch_bounds__(256) xent_bwd_kernel(const bf16* logits, const int64_t* __restrict__ tgt,
                                                        const float* __restrict__ lse_in,
                                                        const float* __restrict__ gscale, bf16* dlogits, int V,
                                                        int Vp) {
  const int64_t row = blockIdx.x;
  const int64_t t = tgt[row];
  const float lse = lse_in[row];
  const float sc = (t >= 0) ? gscale[0] : 0.f;
  const bf16* lr = logits + row * Vp;
  bf16* dr = dlogits + row * Vp;
  const int Vp8 = Vp >> 3;
  for (int c = threadIdx.x; c < Vp8; c += 256) {
    bf16x8 v = *(const bf16x8*)(lr + c * 8);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = c * 8 + j;
      float p = (col < V) ? __expf((float)v[j] - lse) : 0.f;
      if (col == t) p -= 1.f;
      o[j] = (bf16)(p * sc);
    }
    *(bf16x8*)(dr + c * 8) = o;
  }
}

// Fused softmax cross-entropy forward + backward, one row per block with the whole row held in
// registers (TPB threads x NV 16-B vectors): ONE read of the logits and ONE write of the gradient
// (softmax - onehot) / nvalid over the same buffer, versus a read for the loss plus a read and a
// write for the gradient. The loss backward's incoming scalar is applied afterwards only if it is
// not 1 (xent_rescale_kernel). Rows with a negative target contribute neither loss nor gradient.
// KEEP_E: the sum pass keeps e = exp2(x log2e - M) in the row's own registers (as bf16, over the
// logits it no longer needs) and the gradient pass only scales it by 1 / sum: one exp per element
// instead of two (the gradient is rounded to bf16 anyway; e's own bf16 rounding adds one more ulp).
template <int TPB, int NV, int WPE = 6, bool KEEP_E = false>
__global__ void __launch_bounds__(TPB) __attribute__((amdgpu_waves_per_eu(WPE))) xent_fused_kernel(
    bf16* __restrict__ logits, const int64_t* __restrict__ tgt, const float* __restrict__ nvalid,
    float* __restrict__ loss_out, int V, int Vp) {
  constexpr int NW = TPB / 64;
  __shared__ float red[2][NW];
  __shared__ float tlogit;
  const int64_t row = blockIdx.x;
  bf16* lr = logits + row * Vp;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int Vp8 = Vp >> 3;
  const int64_t t = tgt[row];
  if (tid == 0) tlogit = (t >= 0 && t < V) ? (float)lr[t] : 0.f;
  constexpr float L2E = 1.4426950408889634f;
  bf16x8 v[NV];
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = tid + k * TPB;
    if (c < Vp8) v[k] = *(const bf16x8*)(lr + c * 8);
  }
  float m = -INFINITY;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = tid + k * TPB;
    if (c < Vp8) {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (c * 8 + j < V) m = fmaxf(m, (float)v[k][j]);
    }
  }
  m = wave_max(m);
  if (lane == 0) red[0][wid] = m;
  __syncthreads();
  float M = red[0][0];
#pragma unroll
  for (int i = 1; i < NW; ++i) M = fmaxf(M, red[0][i]);
  const float M2 = M * L2E;
  float sum = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = tid + k * TPB;
    if (c < Vp8) {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        if (c * 8 + j < V) {
          const float e = __builtin_amdgcn_exp2f(fmaf((float)v[k][j], L2E, -M2));
          sum += e;
          if constexpr (KEEP_E) v[k][j] = (bf16)e;
        }
      }
    }
  }
  sum = wave_sum(sum);
  if (lane == 0) red[1][wid] = sum;
  __syncthreads();
  float S = 0.f;
#pragma unroll
  for (int i = 0; i < NW; ++i) S += red[1][i];
  const float lse2 = M2 + __builtin_amdgcn_logf(S);  // log2-domain lse (v_log_f32 is log2)
  const float sc = (t >= 0) ? 1.f / nvalid[0] : 0.f;
  const float invS = 1.f / S;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = tid + k * TPB;
    if (c < Vp8) {
      bf16x8 o;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int col = c * 8 + j;
        float p;
        if constexpr (KEEP_E)
          p = (col < V) ? (float)v[k][j] * invS : 0.f;
        else
          p = (col < V) ? __builtin_amdgcn_exp2f(fmaf((float)v[k][j], L2E, -lse2)) : 0.f;
        if (col == t) p -= 1.f;
        o[j] = (bf16)(p * sc);
      }
      *(bf16x8*)(lr + c * 8) = o;
    }
  }
  if (tid == 0) loss_out[row] = (t >= 0) ? lse2 * (1.f / L2E) - tlogit : 0.f;
}

__global__ void __launch_bounds__(256) xent_rescale_kernel(bf16* __restrict__ d, const float* __restrict__ dloss,
                                                           int64_t n8) {
  const float g = dloss[0];
  if (g == 1.f) return;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    bf16x8 v = *(const bf16x8*)(d + i * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = (bf16)((float)v[j] * g);
    *(bf16x8*)(d + i * 8) = v;
  }
}

}  // namespace vcx

// ============================================================ launchers
using namespace vcx;

#define VCX_LN_DISPATCH(CHV, ...)                     \
  switch (CHV) {                                      \
    case 1: { constexpr int CH = 1; __VA_ARGS__; } break; \
    case 2: { constexpr int CH = 2; __VA_ARGS__; } break; \
    case 3: { constexpr int CH = 3; __VA_ARGS__; } break; \
    case 4: { constexpr int CH = 4; __VA_ARGS__; } break; \
    case 5: case 6: { constexpr int CH = 6; __VA_ARGS__; } break; \
    case 7: case 8: { constexpr int CH = 8; __VA_ARGS__; } break; \
    default: { constexpr int CH = 16; __VA_ARGS__; } break; \
  }

void vcx_ln_fwd(const void* a, const void* b, void* xout, void* y, const void* w, const void* bias, float* mean,
                float* rstd, int R, int C, float eps, int rms, const void* bb, hipStream_t s) {
  // VCX_LN_FWD4=0 keeps the one-row-per-wave kernel below (A/B: profiles/r3_ln_fwd_ab.txt)
  static const bool fwd4 = [] {
    const char* e = getenv("VCX_LN_FWD4");
    return !(e && atoi(e) == 0);
  }();
  if (fwd4 && C % 256 == 0 && C <= 1024) {
    static const int resident = [] {  // 5 waves per SIMD (94 VGPRs at C = 768): 5 blocks of 4 waves per CU
      int dev = 0, n = 256;
      (void)hipGetDevice(&dev);
      (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
      return 5 * n;
    }();
    const int blocks = std::min((R + 3) / 4, resident);
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, (const bf16*)a, (const bf16*)b, (bf16*)xout, (bf16*)y,
                         (const bf16*)w, (const bf16*)bias, mean, rstd, R, C, eps, rms, (const bf16*)bb);
    };
    switch (C / 256) {
      case 1: go(ln_fwd4_kernel<1>); return;
      case 2: go(ln_fwd4_kernel<2>); return;
      case 3: go(ln_fwd4_kernel<3>); return;
      default: go(ln_fwd4_kernel<4>); return;
    }
  }
  const int ch = (C / 8 + 63) / 64;
  dim3 grid((R + 3) / 4);
  VCX_LN_DISPATCH(ch, hipLaunchKernelGGL(ln_fwd_kernel<CH>, grid, dim3(256), 0, s, (const bf16*)a,
                                         (const bf16*)b, (bf16*)xout, (bf16*)y, (const bf16*)w,
                                         (const bf16*)bias, mean, rstd, R, C, eps, rms, (const bf16*)bb));
}


static void colsums(const float* p0, const float* p1, const float* p2, void* o0, void* o1, void* o2, int nout, int P,
                    int C, float* stage, hipStream_t s, int accum_mask = 0) {
  hipLaunchKernelGGL(colsum_stage1_kernel, dim3((C + 63) / 64, VCX_COLSUM_NB, nout), dim3(256), 0, s, p0, p1, p2,
                     stage, P, C);
  hipLaunchKernelGGL(colsum_stage2_kernel, dim3((C + 63) / 64, nout), dim3(64), 0, s, stage, VCX_COLSUM_NB, C,
                     (bf16*)o0, (bf16*)o1, (bf16*)o2, accum_mask);
}

static int bias_gelu_groups(int R) { return R < 1024 ? (R > 0 ? R : 1) : 1024; }

int vcx_bias_gelu_partials(int R) { return bias_gelu_groups(R); }

// threads per block: the largest of 256/128/64 that tiles the F/8 column vectors exactly
static int bias_gelu_tpb(int F) {
  const int F8 = F / 8;
  return F8 % 256 == 0 ? 256 : F8 % 128 == 0 ? 128 : 64;
}

#define VCX_TPB_DISPATCH(tpb, ...) \
  do {                               \
    if (tpb == 256) {                \
      constexpr int TPB = 256;       \
      __VA_ARGS__;                   \
    } else if (tpb == 128) {         \
      constexpr int TPB = 128;       \
      __VA_ARGS__;                   \
    } else {                         \
      constexpr int TPB = 64;        \
      __VA_ARGS__;                   \
    }                                \
  } while (0)

void vcx_bias_gelu_fwd(const void* x, const void* b, void* y, int R, int F, hipStream_t s) {
  const int tpb = bias_gelu_tpb(F);
  dim3 grid((F / 8 + tpb - 1) / tpb, R < 1024 ? (R > 0 ? R : 1) : 1024);
  VCX_TPB_DISPATCH(tpb, hipLaunchKernelGGL(bias_gelu_fwd_kernel<TPB>, grid, dim3(TPB), 0, s, (const bf16*)x,
                                           (const bf16*)b, (bf16*)y, R, F));
}

void vcx_bias_gelu_bwd(const void* x, const void* b, const void* dy, void* dx, float* part, void* db, int R, int F,
                       float* stage, int accumulate, hipStream_t s) {
  const int G = bias_gelu_groups(R);
  const int tpb = bias_gelu_tpb(F);
  dim3 grid((F / 8 + tpb - 1) / tpb, G);
  VCX_TPB_DISPATCH(tpb, hipLaunchKernelGGL(bias_gelu_bwd_kernel<TPB>, grid, dim3(TPB), 0, s, (const bf16*)x,
                                           (const bf16*)b, (const bf16*)dy, (bf16*)dx, part, R, F));
  colsums(part, nullptr, nullptr, db, nullptr, nullptr, 1, G, F, stage, s, accumulate ? 1 : 0);
}

static int ln_bwd_blocks(int R, int C) {
  // enough waves to keep every SIMD busy with several rows in flight (each wave streams ~16 rows);
  // the C = 768 variant holds 3 blocks per CU (140 VGPRs): one full round of 768 blocks, no tail
  const int cap = C == 768 ? 768 : 1024;
  const int g = (R + 3) / 4;
  return g > cap ? cap : g;
}

int vcx_ln_bwd_partials(int R, int C) {
  // [P, C] fp32 partial rows: one per block when the row fits the LDS reduction (C <= 2048),
  // else one per wave
  const int ch = (C / 8 + 63) / 64;
  return ch <= 4 ? ln_bwd_blocks(R, C) : ln_bwd_blocks(R, C) * 4;
}

void vcx_ln_bwd(const void* dy, const void* x, const void* w, const float* mean, const float* rstd, const void* dres,
                void* dx, float* dw_part, float* db_part, void* dw, void* db, int R, int C, int rms, float* dbb_part,
                void* dbb, float* stage, int accum_mask, hipStream_t s) {
  const int ch = (C / 8 + 63) / 64;
  const int P = vcx_ln_bwd_partials(R, C);
  dim3 grid(ln_bwd_blocks(R, C));
  if (C == 768) {  // GPT-2-small width: 8-B accesses, 3 per lane (see the kernel)
    if (dres)
      hipLaunchKernelGGL((ln_bwd_kernel<3, true, 4>), grid, dim3(256), 0, s, (const bf16*)dy, (const bf16*)x,
                         (const bf16*)w, mean, rstd, (const bf16*)dres, (bf16*)dx, dw_part, db_part, R, C, rms,
                         dbb_part);
    else
      hipLaunchKernelGGL((ln_bwd_kernel<3, false, 4>), grid, dim3(256), 0, s, (const bf16*)dy, (const bf16*)x,
                         (const bf16*)w, mean, rstd, (const bf16*)nullptr, (bf16*)dx, dw_part, db_part, R, C, rms,
                         dbb_part);
  } else if (dres) {
    VCX_LN_DISPATCH(ch, hipLaunchKernelGGL((ln_bwd_kernel<CH, true, 8>), grid, dim3(256), 0, s, (const bf16*)dy,
                                           (const bf16*)x, (const bf16*)w, mean, rstd, (const bf16*)dres,
                                           (bf16*)dx, dw_part, db_part, R, C, rms, dbb_part));
  } else {
    VCX_LN_DISPATCH(ch, hipLaunchKernelGGL((ln_bwd_kernel<CH, false, 8>), grid, dim3(256), 0, s, (const bf16*)dy,
                                           (const bf16*)x, (const bf16*)w, mean, rstd, (const bf16*)nullptr,
                                           (bf16*)dx, dw_part, db_part, R, C, rms, dbb_part));
  }
  // dw, then db and dbb when present, in one pair of launches; accum_mask bit 0/1/2 = add dw/db/dbb
  // into the existing output (a view of the flat gradient buffer) instead of overwriting it
  const float* ps[3] = {dw_part, nullptr, nullptr};
  void* os[3] = {dw, nullptr, nullptr};
  int slot_mask = accum_mask & 1;
  int n = 1;
  if (db_part && db) {
    slot_mask |= ((accum_mask >> 1) & 1) << n;
    ps[n] = db_part;
    os[n++] = db;
  }
  if (dbb_part && dbb) {
    slot_mask |= ((accum_mask >> 2) & 1) << n;
    ps[n] = dbb_part;
    os[n++] = dbb;
  }
  colsums(ps[0], ps[1], ps[2], os[0], os[1], os[2], n, P, C, stage, s, slot_mask);
}

void vcx_colsum_f32(const float* part, void* out, int P, int C, int accumulate, float* stage, hipStream_t s) {
  colsums(part, nullptr, nullptr, out, nullptr, nullptr, 1, P, C, stage, s, accumulate ? 1 : 0);
}

void vcx_colsum_bf16(const void* y, float* part, void* out, int R, int F, int accumulate, float* stage,
                     hipStream_t s) {
  const int G = bias_gelu_groups(R);
  const int tpb = bias_gelu_tpb(F);
  dim3 grid((F / 8 + tpb - 1) / tpb, G);
  VCX_TPB_DISPATCH(tpb, hipLaunchKernelGGL(colsum_part_bf16_kernel<TPB>, grid, dim3(TPB), 0, s, (const bf16*)y, part,
                                           R, F));
  colsums(part, nullptr, nullptr, out, nullptr, nullptr, 1, G, F, stage, s, accumulate ? 1 : 0);
}

void vcx_gelu_fwd(const void* x, void* y, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(gelu_fwd_kernel, dim3(stream_grid(n / 8, 256)), dim3(256), 0, s, (const bf16*)x, (bf16*)y,
                     n / 8);
}

void vcx_gelu_bwd(const void* x, const void* dy, void* dx, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(gelu_bwd_kernel, dim3(stream_grid(n / 8, 256)), dim3(256), 0, s, (const bf16*)x,
                     (const bf16*)dy, (bf16*)dx, n / 8);
}

void vcx_swiglu_fwd(const void* gu, void* y, int64_t R, int F, hipStream_t s) {
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(stream_grid(R * (F / 8), 256)), dim3(256), 0, s, (const bf16*)gu,
                     (bf16*)y, R, F);
}

void vcx_swiglu_bwd(const void* gu, const void* dy, void* dgu, int64_t R, int F, hipStream_t s) {
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(stream_grid(R * (F / 8), 256)), dim3(256), 0, s, (const bf16*)gu,
                     (const bf16*)dy, (bf16*)dgu, R, F);
}

void vcx_xent_fwd(const void* logits, const int64_t* tgt, float* lse, float* loss, int64_t R, int V, int Vp,
                  hipStream_t s) {
  hipLaunchKernelGGL(xent_fwd_kernel, dim3(R), dim3(256), 0, s, (const bf16*)logits, tgt, lse, loss, V, Vp);
}

void vcx_xent_bwd(const void* logits, const int64_t* tgt, const float* lse, const float* gscale, void* dlogits,
                  int64_t R, int V, int Vp, hipStream_t s) {
  hipLaunchKernelGGL(xent_bwd_kernel, dim3(R), dim3(256), 0, s, (const bf16*)logits, tgt, lse, gscale,
                     (bf16*)dlogits, V, Vp);
}

// returns 0 if the row does not fit the register-resident fused kernel (caller falls back)
int vcx_xent_fused(void* logits, const int64_t* tgt, const float* nvalid, float* loss, int64_t R, int V, int Vp,
                   hipStream_t s) {
  // two rows in flight per CU (12 waves each at <= 85 VGPRs): one row's loads overlap the
  // other's reductions and stores
  const int Vp8 = Vp / 8;
  dim3 grid(R);
  // VCX_XENT_TPB=256 / 512: more, smaller row blocks per CU (4-5 rows in flight per CU instead of
  // 2, each thread holding more of its row); A/B in profiles/r3_xent_variants.txt
  static const int tpb = [] {
    const char* e = getenv("VCX_XENT_TPB");
    return e ? atoi(e) : 768;
  }();
  if (tpb == 256 && Vp8 <= 256 * 25) {
    hipLaunchKernelGGL((xent_fused_kernel<256, 25, 4>), grid, dim3(256), 0, s, (bf16*)logits, tgt, nvalid, loss, V, Vp);
    return 1;
  }
  if (tpb == 512 && Vp8 <= 512 * 13) {
    hipLaunchKernelGGL((xent_fused_kernel<512, 13, 5>), grid, dim3(512), 0, s, (bf16*)logits, tgt, nvalid, loss, V, Vp);
    return 1;
  }
  // one exp per element (KEEP_E above) by default: 2435 vs 2477 us per call at 65536 x 50304, lower max error
  // (scripts/xent_ab.py, gpurun_out/i/xent_*.log); VCX_XENT_KEEP_E=0 restores two
  static const bool keep_e = [] {
    const char* e = getenv("VCX_XENT_KEEP_E");
    return !(e && atoi(e) == 0);
  }();
  if (Vp8 <= 768 * 4)
    hipLaunchKernelGGL((xent_fused_kernel<768, 4>), grid, dim3(768), 0, s, (bf16*)logits, tgt, nvalid, loss, V, Vp);
  else if (Vp8 <= 768 * 9 && keep_e)
    hipLaunchKernelGGL((xent_fused_kernel<768, 9, 6, true>), grid, dim3(768), 0, s, (bf16*)logits, tgt, nvalid, loss,
                       V, Vp);
  else if (Vp8 <= 768 * 9)
    hipLaunchKernelGGL((xent_fused_kernel<768, 9>), grid, dim3(768), 0, s, (bf16*)logits, tgt, nvalid, loss, V, Vp);
  else
    return 0;
  return 1;
}

void vcx_xent_rescale(void* d, const float* dloss, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(xent_rescale_kernel, dim3(stream_grid(n / 8, 256)), dim3(256), 0, s, (bf16*)d, dloss, n / 8);
}
