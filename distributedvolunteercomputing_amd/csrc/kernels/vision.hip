// MobileNet-SSD inference kernels for gfx950 (reference: OpenCV DNN running
// MobileNetSSD_deploy.prototxt on CPU, /root/reference/worker.py:185-280).
//
// Activations are NHWC bf16 for the whole network so that
//   * every 1x1 convolution is a plain GEMM  Y[M=N*H*W, Cout] = X[M, Cin] . W[Cout, Cin]^T,
//     run on MFMA (v_mfma_f32_16x16x32_bf16) with a fused bias+ReLU epilogue;
//   * the depthwise 3x3 convolutions read 16-B channel vectors (8 channels per lane);
//   * the SSD heads' Permute(0,2,3,1)+Flatten is the identity on NHWC data.
// A whole 100-frame chunk is one batch, which turns the per-frame GEMVs of the reference into
// real GEMMs (M = 100*19*19 = 36100 rows for conv11).
#include <algorithm>
#include <cstdlib>

#include "vcx_common.h"

namespace vcx {

// =====================================================================================
// K1+K2+K3: preprocessing
// =====================================================================================
// (a) area (box-filter) resize uint8 BGR [N,H,W,3] -> [N,h,w,3] — imutils.resize(width=400)
//     uses cv2.INTER_AREA; for upscaling INTER_AREA behaves bilinearly, handled by (b).
// INTER_AREA, one thread per output pixel walking its 2-D footprint with global byte loads.
// Measured alternatives (100 x 720p -> 400 px, MI355X): a banded separable kernel with the
// input rows staged in LDS by 16-B loads ran 268 us and the same without LDS 233 us, against
// 188 us for this one (the per-pixel footprints barely overlap, so L1/TA absorb the byte loads).
// The job avoids the cost on the worker side: requesters pre-resize before sending.
__global__ void __launch_bounds__(256) resize_area_u8_kernel(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst,
                                                              int N, int H, int W, int h, int w) {
  const int64_t total = (int64_t)N * h * w;
  const float sx = (float)W / w, sy = (float)H / h;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int x = (int)(i % w);
    const int y = (int)((i / w) % h);
    const int n = (int)(i / ((int64_t)w * h));
    const float fx0 = x * sx, fx1 = fminf((x + 1) * sx, (float)W);
    const float fy0 = y * sy, fy1 = fminf((y + 1) * sy, (float)H);
    float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, wsum = 0.f;
    const uint8_t* base = src + (int64_t)n * H * W * 3;
    for (int yy = (int)fy0; yy < (int)ceilf(fy1) && yy < H; ++yy) {
      const float wy = fminf(fy1, (float)(yy + 1)) - fmaxf(fy0, (float)yy);
      if (wy <= 0.f) continue;
      for (int xx = (int)fx0; xx < (int)ceilf(fx1) && xx < W; ++xx) {
        const float wx = fminf(fx1, (float)(xx + 1)) - fmaxf(fx0, (float)xx);
        if (wx <= 0.f) continue;
        const float wgt = wx * wy;
        const uint8_t* p = base + ((int64_t)yy * W + xx) * 3;
        acc0 = fmaf(wgt, (float)p[0], acc0);
        acc1 = fmaf(wgt, (float)p[1], acc1);
        acc2 = fmaf(wgt, (float)p[2], acc2);
        wsum += wgt;
      }
    }
    const float inv = 1.f / wsum;
    uint8_t* q = dst + i * 3;
    q[0] = (uint8_t)fminf(255.f, fmaxf(0.f, rintf(acc0 * inv)));
    q[1] = (uint8_t)fminf(255.f, fmaxf(0.f, rintf(acc1 * inv)));
    q[2] = (uint8_t)fminf(255.f, fmaxf(0.f, rintf(acc2 * inv)));
  }
}

// (a') the same INTER_AREA as a row-band kernel: one workgroup per (image, output row) stages
//      the input rows of its footprint in LDS with coalesced 16-B loads (every input byte is read
//      from HBM once, plus the fractional rows two bands share) and each thread reduces the
//      footprints of its output pixels from LDS, rows weighted by their vertical overlap.
//      Requires (W*3) % 16 == 0 (1280/1920/640-wide video), w <= RA_XMAX*256 and one input row
//      <= RA_LDS bytes; the launcher falls back to (a) otherwise.
constexpr int RA_LDS = 24 * 1024, RA_XMAX = 4;
// Each thread's output columns are fixed for the whole image, so their horizontal footprints
// (first input column + up to RA_TAPS weights, zero past the footprint) are computed once into
// registers; every row is then a branch-free weighted sum over LDS bytes. (The per-row
// footprint walk with data-dependent trip counts ran 605 instructions per thread, 1.2 TB/s.)
template <int RA_TAPS>
__global__ void __launch_bounds__(256) resize_area_rows_kernel(const uint8_t* __restrict__ src,
                                                                uint8_t* __restrict__ dst, int N, int H, int W, int h,
                                                                int w, float sx, float sy) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[RA_LDS + 1024];  // + a wave's tail lanes
  const int tid = threadIdx.x;
  const int y = blockIdx.x % h, n = blockIdx.x / h;
  const float fy0 = y * sy, fy1 = fminf((y + 1) * sy, (float)H);
  const int iy0 = (int)fy0, iy1 = min((int)ceilf(fy1), H);
  const int rb = W * 3, rpp = RA_LDS / rb;
  int cx0[RA_XMAX];
  float wx[RA_XMAX][RA_TAPS], inv[RA_XMAX];
#pragma unroll
  for (int j = 0; j < RA_XMAX; ++j) {
    const int x = min(tid + 256 * j, w - 1);
    const float fx0 = x * sx, fx1 = fminf((x + 1) * sx, (float)W);
    const int x0 = (int)fx0;
    cx0[j] = min(x0, W - RA_TAPS > 0 ? W - RA_TAPS : 0);  // window start kept inside the row
#pragma unroll
    for (int t = 0; t < RA_TAPS; ++t) {
      const int xx = cx0[j] + t;
      wx[j][t] = fmaxf(0.f, fminf(fx1, (float)(xx + 1)) - fmaxf(fx0, (float)xx));
    }
    inv[j] = 1.f / ((fx1 - fx0) * (fy1 - fy0));
  }
  float acc[RA_XMAX][3];
#pragma unroll
  for (int j = 0; j < RA_XMAX; ++j) acc[j][0] = acc[j][1] = acc[j][2] = 0.f;
  for (int r0 = iy0; r0 < iy1; r0 += rpp) {
    const int nr = min(rpp, iy1 - r0);
    __syncthreads();  // the previous pass has finished reading the band
    // the band's rows straight into LDS (global_load_lds, 16 B per lane): all in flight at once
    const uint8_t* g = src + ((int64_t)n * H + r0) * rb;
    const int chunks = nr * rb / 16;
    for (int e0 = (tid & ~63); e0 < chunks; e0 += 256) {
      const int e = min(e0 + (tid & 63), chunks - 1);  // tail lanes re-copy the last chunk
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + (int64_t)e * 16),
                                       (__attribute__((address_space(3))) void*)(rows + e0 * 16), 16, 0, 0);
    }
    __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
    __syncthreads();
    for (int r = 0; r < nr; ++r) {
      const float wy = fmaxf(0.f, fminf(fy1, (float)(r0 + r + 1)) - fmaxf(fy0, (float)(r0 + r)));
      const uint8_t* row = rows + r * rb;
#pragma unroll
      for (int j = 0; j < RA_XMAX; ++j) {
        if (256 * j >= w) break;  // uniform
        float h0 = 0.f, h1 = 0.f, h2 = 0.f;
        const uint8_t* p = row + cx0[j] * 3;
#pragma unroll
        for (int t = 0; t < RA_TAPS; ++t) {
          h0 = fmaf(wx[j][t], (float)p[3 * t], h0);
          h1 = fmaf(wx[j][t], (float)p[3 * t + 1], h1);
          h2 = fmaf(wx[j][t], (float)p[3 * t + 2], h2);
        }
        acc[j][0] = fmaf(wy, h0, acc[j][0]);
        acc[j][1] = fmaf(wy, h1, acc[j][1]);
        acc[j][2] = fmaf(wy, h2, acc[j][2]);
      }
    }
  }
  uint8_t* q = dst + ((int64_t)n * h + y) * w * 3;
#pragma unroll
  for (int j = 0; j < RA_XMAX; ++j) {
    const int x = tid + 256 * j;
    if (x >= w) break;
#pragma unroll
    for (int c = 0; c < 3; ++c) q[x * 3 + c] = (uint8_t)fminf(255.f, fmaxf(0.f, rintf(acc[j][c] * inv[j])));
  }
}

// (b) bilinear (half-pixel centres, cv2.INTER_LINEAR) uint8 [N,H,W,3] -> uint8 [N,h,w,3]
__global__ void __launch_bounds__(256) resize_bilinear_u8_kernel(const uint8_t* __restrict__ src,
                                                                  uint8_t* __restrict__ dst, int N, int H, int W,
                                                                  int h, int w) {
  const int64_t total = (int64_t)N * h * w;
  const float sx = (float)W / w, sy = (float)H / h;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int x = (int)(i % w), y = (int)((i / w) % h), n = (int)(i / ((int64_t)w * h));
    float fx = fmaxf((x + 0.5f) * sx - 0.5f, 0.f), fy = fmaxf((y + 0.5f) * sy - 0.5f, 0.f);
    int x0 = min((int)fx, W - 1), y0 = min((int)fy, H - 1);
    int x1 = min(x0 + 1, W - 1), y1 = min(y0 + 1, H - 1);
    float ax = fx - x0, ay = fy - y0;
    const uint8_t* b = src + (int64_t)n * H * W * 3;
    for (int c = 0; c < 3; ++c) {
      float v00 = b[((int64_t)y0 * W + x0) * 3 + c], v01 = b[((int64_t)y0 * W + x1) * 3 + c];
      float v10 = b[((int64_t)y1 * W + x0) * 3 + c], v11 = b[((int64_t)y1 * W + x1) * 3 + c];
      float v = (v00 * (1 - ax) + v01 * ax) * (1 - ay) + (v10 * (1 - ax) + v11 * ax) * ay;
      dst[i * 3 + c] = (uint8_t)fminf(255.f, fmaxf(0.f, rintf(v)));
    }
  }
}

// (c) cv2.resize(frame, (S,S)) bilinear -> blobFromImage(scale, mean) -> NHWC bf16, channel
//     padded to CP (=4) lanes with zeros: [N, S, S, CP]. BGR order kept (no swapRB).
//     3-D grid: blockIdx.z = image, blockIdx.y = output row, so the source rows and vertical weights are
//     scalar; one thread per output column (the grid-stride version with 64-bit index division
//     per pixel ran at 1.7 TB/s).
constexpr int BLOB_LDS = 12 * 1024;  // two source rows of up to 2048 px
__global__ void __launch_bounds__(320) blob_bilinear_kernel(const uint8_t* __restrict__ src, bf16* __restrict__ dst,
                                                             int N, int H, int W, int S, float sx, float sy,
                                                             float scale, float mean) {
  __shared__ __attribute__((aligned(16))) uint8_t rows[2 * BLOB_LDS + 1024];
  const int tid = threadIdx.x;
  const int n = blockIdx.z, y = blockIdx.y;
  const float fy = fmaxf((y + 0.5f) * sy - 0.5f, 0.f);
  const int y0 = min((int)fy, H - 1), y1 = min(y0 + 1, H - 1);
  const float ay = fy - y0;
  const int rb = W * 3;
  // the two source rows into LDS (16-B LDS-DMA; row bytes are a multiple of 16, host-checked),
  // so each output pixel's 12 byte taps are LDS reads instead of 12 global byte loads
  const int chunks = rb / 16;
  for (int rr = 0; rr < 2; ++rr) {
    const uint8_t* g = src + ((int64_t)n * H + (rr ? y1 : y0)) * rb;
    for (int e0 = (tid & ~63); e0 < chunks; e0 += blockDim.x) {
      const int e = min(e0 + (tid & 63), chunks - 1);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + (int64_t)e * 16),
                                       (__attribute__((address_space(3))) void*)(rows + rr * BLOB_LDS + e0 * 16), 16,
                                       0, 0);
    }
  }
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
  __syncthreads();
  for (int x = blockIdx.x * blockDim.x + tid; x < S; x += gridDim.x * blockDim.x) {
    const float fx = fmaxf((x + 0.5f) * sx - 0.5f, 0.f);
    const int x0 = min((int)fx, W - 1), x1 = min(x0 + 1, W - 1);
    const float ax = fx - x0;
    const uint8_t* r0 = rows;
    const uint8_t* r1 = rows + BLOB_LDS;
    bf16x4 o;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      const float v00 = r0[x0 * 3 + c], v01 = r0[x1 * 3 + c], v10 = r1[x0 * 3 + c], v11 = r1[x1 * 3 + c];
      float v = (v00 * (1 - ax) + v01 * ax) * (1 - ay) + (v10 * (1 - ax) + v11 * ax) * ay;
      v = rintf(fminf(255.f, fmaxf(0.f, v)));  // cv2.resize output is uint8
      o[c] = (bf16)((v - mean) * scale);
    }
    o[3] = (bf16)0.f;
    *(bf16x4*)(dst + (((int64_t)n * S + y) * S + x) * 4) = o;
  }
}

// RB output rows per workgroup: the source rows they need (consecutive in memory: one linear
// LDS-DMA copy of at most (RB - 1) * sy + 3 rows) are loaded once and shared, instead of two source
// rows per one-row workgroup (each source row was fetched ~2.7 times at 225 -> 300, and a 2.4 KB
// row of output per workgroup left too few bytes in flight: 2.2 TB/s).
template <int RB>
__global__ void __launch_bounds__(320) blob_bilinear_rows_kernel(const uint8_t* __restrict__ src,
                                                                  bf16* __restrict__ dst, int N, int H, int W, int S,
                                                                  float sx, float sy, float scale, float mean) {
  extern __shared__ __attribute__((aligned(16))) uint8_t brows[];
  const int tid = threadIdx.x;
  const int n = blockIdx.z, yb = blockIdx.y * RB, ye = min(yb + RB, S);
  const int rb = W * 3;
  auto row0 = [&](int y) { return min((int)fmaxf((y + 0.5f) * sy - 0.5f, 0.f), H - 1); };
  const int ry0 = row0(yb), ry1 = min(row0(ye - 1) + 1, H - 1);
  const int chunks = (ry1 - ry0 + 1) * rb / 16;
  const uint8_t* g = src + ((int64_t)n * H + ry0) * rb;
  for (int e0 = (tid & ~63); e0 < chunks; e0 += blockDim.x) {
    const int e = min(e0 + (tid & 63), chunks - 1);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + (int64_t)e * 16),
                                     (__attribute__((address_space(3))) void*)(brows + e0 * 16), 16, 0, 0);
  }
  __builtin_amdgcn_s_waitcnt(0x0070);  // vmcnt(0) lgkmcnt(0)
  __syncthreads();
  for (int y = yb; y < ye; ++y) {
    const float fy = fmaxf((y + 0.5f) * sy - 0.5f, 0.f);
    const int y0 = min((int)fy, H - 1), y1 = min(y0 + 1, H - 1);
    const float ay = fy - y0;
    const uint8_t* r0 = brows + (y0 - ry0) * rb;
    const uint8_t* r1 = brows + (y1 - ry0) * rb;
    for (int x = tid; x < S; x += blockDim.x) {
      const float fx = fmaxf((x + 0.5f) * sx - 0.5f, 0.f);
      const int x0 = min((int)fx, W - 1), x1 = min(x0 + 1, W - 1);
      const float ax = fx - x0;
      bf16x4 o;
#pragma unroll
      for (int c = 0; c < 3; ++c) {
        const float v00 = r0[x0 * 3 + c], v01 = r0[x1 * 3 + c], v10 = r1[x0 * 3 + c], v11 = r1[x1 * 3 + c];
        float v = (v00 * (1 - ax) + v01 * ax) * (1 - ay) + (v10 * (1 - ax) + v11 * ax) * ay;
        v = rintf(fminf(255.f, fmaxf(0.f, v)));
        o[c] = (bf16)((v - mean) * scale);
      }
      o[3] = (bf16)0.f;
      *(bf16x4*)(dst + (((int64_t)n * S + y) * S + x) * 4) = o;
    }
  }
}

// the same for widths whose rows are not 16-B multiples (global byte taps)
__global__ void __launch_bounds__(256) blob_bilinear_any_kernel(const uint8_t* __restrict__ src,
                                                                 bf16* __restrict__ dst, int N, int H, int W, int S,
                                                                 float sx, float sy, float scale, float mean) {
  const int x = blockIdx.x * blockDim.x + threadIdx.x;
  if (x >= S) return;
  const int n = blockIdx.z, y = blockIdx.y;
  const float fy = fmaxf((y + 0.5f) * sy - 0.5f, 0.f);
  const int y0 = min((int)fy, H - 1), y1 = min(y0 + 1, H - 1);
  const float ay = fy - y0;
  const float fx = fmaxf((x + 0.5f) * sx - 0.5f, 0.f);
  const int x0 = min((int)fx, W - 1), x1 = min(x0 + 1, W - 1);
  const float ax = fx - x0;
  const uint8_t* r0 = src + ((int64_t)n * H + y0) * W * 3;
  const uint8_t* r1 = src + ((int64_t)n * H + y1) * W * 3;
  bf16x4 o;
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float v00 = r0[x0 * 3 + c], v01 = r0[x1 * 3 + c], v10 = r1[x0 * 3 + c], v11 = r1[x1 * 3 + c];
    float v = (v00 * (1 - ax) + v01 * ax) * (1 - ay) + (v10 * (1 - ax) + v11 * ax) * ay;
    v = rintf(fminf(255.f, fmaxf(0.f, v)));
    o[c] = (bf16)((v - mean) * scale);
  }
  o[3] = (bf16)0.f;
  *(bf16x4*)(dst + (((int64_t)n * S + y) * S + x) * 4) = o;
}

// =====================================================================================
// im2col for dense KxK convolutions on NHWC bf16 (stem conv0 and the SSD extras' 3x3 s2)
// out[m, k] with m = (n, oy, ox), k = (ky, kx, c) for c < C (channel stride Cs), zero-padded
// to Kp columns (Kp % 32 == 0).
// =====================================================================================
__global__ void __launch_bounds__(256) im2col_nhwc_kernel(const bf16* __restrict__ x, bf16* __restrict__ out, int N,
                                                           int H, int W, int C, int Cs, int Ho, int Wo, int KH,
                                                           int KW, int stride, int pad, int Kp) {
  const int64_t total = (int64_t)N * Ho * Wo * Kp;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int k = (int)(i % Kp);
    const int64_t m = i / Kp;
    const int ox = (int)(m % Wo), oy = (int)((m / Wo) % Ho), n = (int)(m / ((int64_t)Wo * Ho));
    bf16 v = (bf16)0.f;
    if (k < KH * KW * C) {
      const int c = k % C, kx = (k / C) % KW, ky = k / (C * KW);
      const int iy = oy * stride - pad + ky, ix = ox * stride - pad + kx;
      if (iy >= 0 && iy < H && ix >= 0 && ix < W) v = x[(((int64_t)n * H + iy) * W + ix) * Cs + c];
    }
    out[i] = v;
  }
}

// =====================================================================================
// K5: depthwise 3x3 conv + bias + ReLU, NHWC bf16, stride 1|2, pad 1. 8 channels per lane.
// The 9-tap reduction runs on v_dot2_f32_bf16: taps (2p, 2p+1) of one channel are paired with
// one v_perm_b32 and reduced with their paired weights in one dot2 (4 pairs + the 9th tap against
// (w8, 0) / (0, w8)): 9 VALU ops per output instead of 9 FMAs plus 18 bf16->fp32 unpacks — the
// fp32 version was VALU-bound (r2: 40.7 us per layer at 2.85 TB/s).
// Paired weights wp: [5][C] dwords, wp[p][c] = (w[2p][c], w[2p+1][c]) for p < 4,
// wp[4][c] = (w[8][c], 0) for even c and (0, w[8][c]) for odd c (ops/vision.py dw_pair_weights).
// =====================================================================================
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot2bf(uint32_t a, uint32_t b, float c) {
  return __builtin_amdgcn_fdot2_f32_bf16(__builtin_bit_cast(bf16x2v, a), __builtin_bit_cast(bf16x2v, b), c, false);
}

// a[j] += sum_t x[t][j] * w[t][j] for the 8 channels of one lane; wp -> paired weights of the
// first of those channels, ldw = dwords between pair rows (C)
__device__ __forceinline__ void dw9_accum(const u32x4 (&x)[9], const uint32_t* wp, int ldw, float (&a)[8]) {
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    const u32x4 w0 = *(const u32x4*)(wp + p * ldw), w1 = *(const u32x4*)(wp + p * ldw + 4);
    const uint32_t w[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t lo = x[2 * p][q], hi = x[2 * p + 1][q];
      a[2 * q] = dot2bf(__builtin_amdgcn_perm(hi, lo, 0x05040100u), w[2 * q], a[2 * q]);
      a[2 * q + 1] = dot2bf(__builtin_amdgcn_perm(hi, lo, 0x07060302u), w[2 * q + 1], a[2 * q + 1]);
    }
  }
  const u32x4 w0 = *(const u32x4*)(wp + 4 * ldw), w1 = *(const u32x4*)(wp + 4 * ldw + 4);
  const uint32_t w[8] = {w0[0], w0[1], w0[2], w0[3], w1[0], w1[1], w1[2], w1[3]};
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[2 * q] = dot2bf(x[8][q], w[2 * q], a[2 * q]);
    a[2 * q + 1] = dot2bf(x[8][q], w[2 * q + 1], a[2 * q + 1]);
  }
}

// the same with the paired weights of the lane's 8 channels already in registers (w[p][j])
__device__ __forceinline__ void load_dw_weights(const uint32_t* wp, int ldw, uint32_t (&w)[5][8]) {
#pragma unroll
  for (int p = 0; p < 5; ++p) {
    const u32x4 w0 = *(const u32x4*)(wp + p * ldw), w1 = *(const u32x4*)(wp + p * ldw + 4);
    w[p][0] = w0[0], w[p][1] = w0[1], w[p][2] = w0[2], w[p][3] = w0[3];
    w[p][4] = w1[0], w[p][5] = w1[1], w[p][6] = w1[2], w[p][7] = w1[3];
  }
}
__device__ __forceinline__ void dw9_accum_w(const u32x4 (&x)[9], const uint32_t (&w)[5][8], float (&a)[8]) {
#pragma unroll
  for (int p = 0; p < 4; ++p)
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t lo = x[2 * p][q], hi = x[2 * p + 1][q];
      a[2 * q] = dot2bf(__builtin_amdgcn_perm(hi, lo, 0x05040100u), w[p][2 * q], a[2 * q]);
      a[2 * q + 1] = dot2bf(__builtin_amdgcn_perm(hi, lo, 0x07060302u), w[p][2 * q + 1], a[2 * q + 1]);
    }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    a[2 * q] = dot2bf(x[8][q], w[4][2 * q], a[2 * q]);
    a[2 * q + 1] = dot2bf(x[8][q], w[4][2 * q + 1], a[2 * q + 1]);
  }
}

__device__ __forceinline__ u32x4 dw_out8(const float (&a)[8], int relu) {
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o[j] = (bf16)(relu ? fmaxf(a[j], 0.f) : a[j]);
  return __builtin_bit_cast(u32x4, o);
}

// One thread = one (column ox, 8-channel group) and R consecutive output rows: the (R-1)*stride+3
// input rows x 3 columns it needs are ALL loaded before any reduction (R = 4 at stride 1: 18
// loads for 4 outputs instead of 36, and every wave keeps 18 KB of loads in flight, most of it
// L1/L2 hits around ~3 KB of new HBM data). 2-D grid: blockIdx.y = (image, row group) so the
// image/row split is scalar; lanes run along (ox, c8) with C8 a power of two (a shift). The
// previous grid-stride version (one output per iteration, 64-bit index division) measured
// 135 us for conv1/dw (288 MB, 2.1 TB/s).
template <int STRIDE, int R>
__global__ void __launch_bounds__(256) dwconv3x3_kernel(const bf16* __restrict__ x, const uint32_t* __restrict__ wp,
                                                         const float* __restrict__ b, bf16* __restrict__ y, int H,
                                                         int W, int C, int Ho, int Wo, int c8_shift, int relu) {
  constexpr int NR = (R - 1) * STRIDE + 3;  // input rows per thread
  const int C8 = C >> 3;
  const int idx = blockIdx.x * 256 + threadIdx.x;
  const int ox = c8_shift >= 0 ? idx >> c8_shift : idx / C8;  // (C8 not a power of two: a divide)
  const int c8 = idx - ox * C8;
  if (ox >= Wo) return;
  const int groups = (Ho + R - 1) / R;
  const int n = blockIdx.y / groups, oy0 = (blockIdx.y - n * groups) * R;
  const int iy0 = oy0 * STRIDE - 1, ix0 = ox * STRIDE - 1;
  // taps through a buffer resource over this image: rows above/below the image fall outside the
  // resource and read as zero (the pad), so only the left/right pad columns need a mask
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)n * H * W * C), (short)0,
                                                    H * W * C * 2, 0x00020000);
  const int rowb = W * C * 2, pixb = C * 2;
  const int base = (iy0 * W + ix0) * pixb + c8 * 16;
  int coff[3];
#pragma unroll
  for (int kx = 0; kx < 3; ++kx) coff[kx] = (ix0 + kx >= 0 && ix0 + kx < W) ? base + kx * pixb : (int)0x80000000;
  u32x4 xv[NR][3];
#pragma unroll
  for (int r = 0; r < NR; ++r)
#pragma unroll
    for (int kx = 0; kx < 3; ++kx)
      xv[r][kx] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, coff[kx] + r * rowb, 0, 0));
  f32x4 b0 = *(const f32x4*)(b + c8 * 8), b1 = *(const f32x4*)(b + c8 * 8 + 4);
  // the weights once per thread, in registers: reloading them per output row (the loop's early
  // exit keeps the compiler from hoisting) tripled the L1 traffic — 40 weight loads against 18
  // tap loads per thread, and the kernel ran L1/TA-bound at 2.7 TB/s
  uint32_t wr[5][8];
  load_dw_weights(wp + c8 * 8, C, wr);
#pragma unroll
  for (int j = 0; j < R; ++j) {
    const int oy = oy0 + j;
    if (oy >= Ho) break;
    float acc[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    const u32x4 t9[9] = {xv[j * STRIDE][0],     xv[j * STRIDE][1],     xv[j * STRIDE][2],
                         xv[j * STRIDE + 1][0], xv[j * STRIDE + 1][1], xv[j * STRIDE + 1][2],
                         xv[j * STRIDE + 2][0], xv[j * STRIDE + 2][1], xv[j * STRIDE + 2][2]};
    dw9_accum_w(t9, wr, acc);
    *(u32x4*)(y + (((int64_t)n * Ho + oy) * Wo + ox) * C + c8 * 8) = dw_out8(acc, relu);
  }
}

// =====================================================================================
// K6/K7/K8: GEMM  Y[M, N] = act(X[M, K] . W[N, K]^T + bias[N])   (bf16 in, fp32 acc, bf16 out)
// Block tile 128 x BN (BN = 128 | 64), BK = 32, 256 threads = 4 waves in a 2 x 2 grid; each
// wave owns a 64 x (BN/2) sub-tile made of 16x16 MFMA tiles (v_mfma_f32_16x16x32_bf16: one
// MFMA per 16x16 tile per K-step). LDS rows are XOR-swizzled 64-B rows (gidx below). Global->LDS
// staging is double-buffered through registers (load tile k+1 while tile k feeds the MFMAs).
// Blocks are remapped so that consecutive tiles of one M panel land on the same XCD (they
// share the X panel through that XCD's L2). Requires K % 32 == 0; M, N arbitrary.
// =====================================================================================
typedef short bf16x8s __attribute__((ext_vector_type(8)));
constexpr int GBM = 128, GBK = 32, GLDK = 32;

// LDS image of a [rows][32] bf16 tile: 64-B rows, 16-B chunks XOR-swizzled by
// F[(row >> 2) & 3] = {0, 2, 3, 1}. Every ds_read_b128 lane group (16 rows, two chunks) then hits
// 16 distinct 16-B bank slots; the former 80-B padded rows measured 5.3 bank conflicts per LDS
// instruction (rocprofv3 SQ_LDS_BANK_CONFLICT / SQ_INSTS_LDS).
__device__ __forceinline__ int gswz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }
__device__ __forceinline__ int gidx(int row, int chunk) { return row * GLDK + ((chunk ^ gswz(row)) << 3); }

// Output mapping (epilogue): row m of image (m / rpi), column n:
//   n <  split: Y  + (m / rpi) * img_stride  + (m % rpi) * ldy  + n
//   n >= split: Y2 + (m / rpi) * img_stride2 + (m % rpi) * ldy2 + (n - split)
// A plain GEMM is rpi = M, split = N. The SSD heads use it to run loc||conf of one source as ONE
// GEMM that writes both straight into the concatenated mbox_loc / mbox_conf buffers (Permute +
// Flatten + Concat, prototxt 1172-1858, become address arithmetic).
struct OutMap {
  bf16* Y2;
  int split, ldy2, rpi;
  int64_t img_stride, img_stride2;
  float* part;  // split-K: fp32 partial sums [gridDim.z][M][N] instead of the epilogue (else null)
  int kchunk;   // split-K: K columns per z (multiple of 32)
  int* cnt;     // split-K: per-tile tickets (zero between launches) -> the last block reduces, or null
};

// split-K reduction + the epilogue (bias, ReLU, bf16, output mapping) for the partials above
__global__ void __launch_bounds__(256) splitk_bias_act_kernel(const float* __restrict__ part, int S,
                                                               const float* __restrict__ bias, bf16* __restrict__ Y,
                                                               int M, int N, int ldy, int relu, OutMap om) {
  const int64_t total = (int64_t)M * N;
  for (int64_t e = blockIdx.x * 256ll + threadIdx.x; e < total; e += (int64_t)gridDim.x * 256) {
    float v = bias ? bias[e % N] : 0.f;
    for (int z = 0; z < S; ++z) v += part[z * total + e];
    if (relu) v = fmaxf(v, 0.f);
    const int gm = (int)(e / N), n = (int)(e - (int64_t)gm * N);
    const int64_t img = gm / om.rpi, rr = gm - img * om.rpi;
    if (n < om.split) Y[img * om.img_stride + rr * ldy + n] = (bf16)v;
    else om.Y2[img * om.img_stride2 + rr * om.ldy2 + (n - om.split)] = (bf16)v;
  }
}

// A-operand modes of the GEMM below:
//  AM_PLAIN    X is the [M, K] activation matrix.
//  AM_IMPLICIT implicit-GEMM convolution: X is the NHWC input [imgs, H, W, Cs] and the A tile
//              row m = (img, oy, ox), column k = (ky, kx, c) is gathered while staging — no
//              im2col matrix is written or read (the stem's was 144 MB per 100-frame chunk).
//              C % 8 == 0: one 16-B load per 8 columns (one tap); C == 4 (the stem's padded BGR0
//              blob): two 8-B loads (two taps).
//  AM_DW       depthwise 3x3 (pad 1, stride 1|2) + bias (+ReLU) fused in front of the pointwise
//              GEMM (SURVEY K5 "optionally fused with the following pointwise GEMM"; prototxt
//              conv1/dw -> conv1 and the 12 pairs after it, MobileNetSSD_deploy.prototxt:42-106):
//              X is the depthwise INPUT [imgs, H, W, K] and each K-slice of the A tile is computed
//              from its 9 taps while staging, so the depthwise output never goes through HBM.
enum { AM_PLAIN = 0, AM_IMPLICIT = 1, AM_DW = 2 };
constexpr int DW_KMAX = 1024;
struct ConvGeom {
  int H, W, C, Cs, Ho, Wo, KW, stride, pad, Kreal;
  const uint32_t* dw_w;  // AM_DW: [5][K] paired depthwise weights (see dw9_accum)
  const float* dw_b;  // AM_DW: [K] depthwise bias
  int dw_relu;
};

template <int BN, int AM>
__global__ void __launch_bounds__(256) gemm_bias_act_kernel(const bf16* __restrict__ X, const bf16* __restrict__ Wt,
                                                             const float* __restrict__ bias, bf16* __restrict__ Y,
                                                             int M, int N, int K, int ldy, int relu, OutMap om,
                                                             ConvGeom cg) {
  // operand ring (2 x A 128x32 + 2 x B BNx32) and, after the main loop, the bf16 output tile
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * GBM * GLDK + 2 * BN * GLDK];
  bf16* const sA0 = smem;
  bf16* const sB0 = smem + 2 * GBM * GLDK;
  constexpr int WN = BN / 2;          // per-wave N extent
  constexpr int TN = WN / 16;         // 16x16 tiles per wave along N
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;
  // AM_DW: paired depthwise weights [5][K] dwords + bias [K] fp32 for the whole K (K <= DW_KMAX)
  __shared__ __attribute__((aligned(16))) uint32_t dw_lds_w[AM == AM_DW ? 5 * DW_KMAX : 4];
  __shared__ __attribute__((aligned(16))) float dw_lds_b[AM == AM_DW ? DW_KMAX : 4];
  if constexpr (AM == AM_DW) {
    for (int e = tid; e < 5 * K / 4; e += 256) ((u32x4*)dw_lds_w)[e] = ((const u32x4*)cg.dw_w)[e];
    for (int e = tid; e < K / 4; e += 256) ((f32x4*)dw_lds_b)[e] = ((const f32x4*)cg.dw_b)[e];
    __syncthreads();
  }

  // XCD-aware, bijective block remap (cdna guide §5 T1): group label = bid % 8
  const int ntm = (M + GBM - 1) / GBM, ntn = (N + BN - 1) / BN;
  const int nwg = ntm * ntn;
  int bid = blockIdx.x;
  {
    const int q = nwg / 8, r = nwg % 8, xcd = bid % 8, idx = bid / 8;
    if (nwg >= 8) bid = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + idx;
  }
  const int tm = bid / ntn, tn = bid % ntn;
  const int m0 = tm * GBM, n0 = tn * BN;

  // staging: A tile 128x32 bf16 = 512 x 16 B -> 2 per thread; B tile BN x 32 -> BN/128 per thread
  constexpr int BL = BN * 4 / 256;  // 16-B loads of B per thread
  bf16x8s ra[2], rb[BL];
  // implicit conv / depthwise: the output pixel of each of this thread's two A rows (fixed)
  int pix_img[2], pix_iy[2], pix_ix[2];
  if constexpr (AM != AM_PLAIN) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int gm = m0 + ((tid + i * 256) >> 2);
      const int hw = cg.Ho * cg.Wo;
      const int img = gm / hw, r = gm - img * hw, oy = r / cg.Wo, ox = r - oy * cg.Wo;
      pix_img[i] = gm < M ? img : -1;
      pix_iy[i] = oy * cg.stride - cg.pad;
      pix_ix[i] = ox * cg.stride - cg.pad;
    }
  }
  auto tap_ptr = [&](int i, int k) -> const bf16* {  // input address of column k for row i, or null
    if (k >= cg.Kreal) return nullptr;
    const int tap = k / cg.C, c = k - tap * cg.C, ky = tap / cg.KW, kx = tap - ky * cg.KW;
    const int iy = pix_iy[i] + ky, ix = pix_ix[i] + kx;
    if (iy < 0 || iy >= cg.H || ix < 0 || ix >= cg.W) return nullptr;
    return X + (((int64_t)pix_img[i] * cg.H + iy) * cg.W + ix) * cg.Cs + c;
  };
  // AM_DW: the 9 taps of both rows of this thread's 8 channels, loaded in gload (in flight during
  // the MFMAs) and reduced in sstore against the depthwise weights, which sit in LDS for the
  // whole K (dw_lds: [9][K] bf16 then [K] fp32 bias; at most 9*1024*2 + 4096 B)
  u32x4 dtap[2][9];
  uint32_t tapok[2] = {0, 0};    // bit t: tap t inside the image
  const bf16* pixbase[2] = {X, X};  // input address of tap 0 (row above, column left)
  if constexpr (AM == AM_DW) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      if (pix_img[i] < 0) continue;
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        const int iy = pix_iy[i] + t / 3, ix = pix_ix[i] + t % 3;
        if (iy >= 0 && iy < cg.H && ix >= 0 && ix < cg.W) tapok[i] |= 1u << t;
      }
      pixbase[i] = X + (((int64_t)pix_img[i] * cg.H + pix_iy[i]) * cg.W + pix_ix[i]) * K;
    }
  }
  auto gload = [&](int k0) {
    if constexpr (AM == AM_DW) {
      const int c = k0 + (tid & 3) * 8;  // the same 8 channels for both rows (256 % 4 == 0)
      const int rowst = cg.W * K;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
#pragma unroll
        for (int t = 0; t < 9; ++t) {
          const int off = (t / 3) * rowst + (t % 3) * K + c;
          dtap[i][t] = (tapok[i] >> t) & 1 ? *(const u32x4*)(pixbase[i] + off) : u32x4{0u, 0u, 0u, 0u};
        }
      }
    } else {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, row = e >> 2, kc = (e & 3) * 8;
        const int gm = m0 + row;
        if constexpr (AM == AM_IMPLICIT) {
          bf16x8s v = bf16x8s{0, 0, 0, 0, 0, 0, 0, 0};
          if (pix_img[i] >= 0) {
            if (cg.C % 8 == 0) {
              const bf16* q = tap_ptr(i, k0 + kc);
              if (q) v = *(const bf16x8s*)q;
            } else {  // C == 4: two taps of 4 channels
              typedef short sx4v __attribute__((ext_vector_type(4)));
              const bf16* q0 = tap_ptr(i, k0 + kc);
              const bf16* q1 = tap_ptr(i, k0 + kc + 4);
              const sx4v a = q0 ? *(const sx4v*)q0 : sx4v{0, 0, 0, 0};
              const sx4v b = q1 ? *(const sx4v*)q1 : sx4v{0, 0, 0, 0};
              v = bf16x8s{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
            }
          }
          ra[i] = v;
        } else {
          ra[i] = gm < M ? *(const bf16x8s*)(X + (int64_t)gm * K + k0 + kc) : bf16x8s{0, 0, 0, 0, 0, 0, 0, 0};
        }
      }
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int e = tid + i * 256, row = e >> 2, kc = (e & 3) * 8;
      const int gn = n0 + row;
      rb[i] = gn < N ? *(const bf16x8s*)(Wt + (int64_t)gn * K + k0 + kc) : bf16x8s{0, 0, 0, 0, 0, 0, 0, 0};
    }
  };
  auto sstore = [&](int buf, int k0) {
    if constexpr (AM == AM_DW) {
      const int c = k0 + (tid & 3) * 8;
      const f32x4 b0 = *(const f32x4*)(dw_lds_b + c), b1 = *(const f32x4*)(dw_lds_b + c + 4);
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        float a[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
        dw9_accum(dtap[i], dw_lds_w + c, K, a);
        // rounded to bf16 exactly where the unfused depthwise kernel writes its output
        ra[i] = __builtin_bit_cast(bf16x8s, dw_out8(a, cg.dw_relu));
      }
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int e = tid + i * 256, row = e >> 2;
      *(bf16x8s*)(&sA0[buf * GBM * GLDK + gidx(row, e & 3)]) = ra[i];
    }
#pragma unroll
    for (int i = 0; i < BL; ++i) {
      const int e = tid + i * 256, row = e >> 2;
      *(bf16x8s*)(&sB0[buf * BN * GLDK + gidx(row, e & 3)]) = rb[i];
    }
  };

  f32x4 acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // split-K (small-M layers, part != nullptr): blockIdx.z takes K columns [kz0, kz0 + kc)
  const int kc = om.part ? om.kchunk : K;
  const int kz0 = om.part ? blockIdx.z * kc : 0;
  const int nk = kc / GBK;
  gload(kz0);
  sstore(0, kz0);
  __syncthreads();
  const int fr = lane & 15, fc = lane >> 4;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gload(kz0 + (kt + 1) * GBK);
    const bf16* sA = sA0 + cur * GBM * GLDK;
    const bf16* sB = sB0 + cur * BN * GLDK;
    bf16x8s af[4], bfr[TN];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8s*)(&sA[gidx(wm * 64 + i * 16 + fr, fc)]);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *(const bf16x8s*)(&sB[gidx(wn * WN + j * 16 + fr, fc)]);
    // operand order W x X: a lane's accumulator holds 4 consecutive output COLUMNS of one row
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    if (kt + 1 < nk) sstore(cur ^ 1, kz0 + (kt + 1) * GBK);
    __syncthreads();
  }

  if (om.part) {  // split-K partial: fp32 accumulators straight out, [z][M][N] (reduced by splitk_bias_act)
    float* const pz = om.part + (int64_t)blockIdx.z * M * N;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int gn = n0 + wn * WN + j * 16 + 4 * (lane >> 4);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int gm = m0 + wm * 64 + i * 16 + (lane & 15);
        if (gm >= M) continue;
        float* q = pz + (int64_t)gm * N + gn;
        if (gn + 3 < N && (N & 3) == 0) {
          *(f32x4*)q = acc[i][j];
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (gn + r < N) q[r] = acc[i][j][r];
        }
      }
    }
    if (!om.cnt) return;  // reduced by splitk_bias_act
    // the LAST of the tile's S blocks reduces it (no separate reduction launch): publish the
    // partial (stores retired, agent-scope release), take a ticket; the block holding the final
    // ticket acquires, sums the S partials of the tile and runs the epilogue; it also re-arms
    // the tile's counter for the next launch (self-resetting, one counter array per stream)
    __shared__ int s_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) {
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      const int t = atomicAdd(om.cnt + blockIdx.x, 1);
      s_last = t == (int)gridDim.z - 1;
      if (s_last) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        atomicExch(om.cnt + blockIdx.x, 0);
      }
    }
    __syncthreads();
    if (!s_last) return;
    const int S = gridDim.z;
    const int64_t MN = (int64_t)M * N;
    for (int e = tid; e < GBM * BN; e += 256) {
      const int gm = m0 + e / BN, n = n0 + e % BN;
      if (gm >= M || n >= N) continue;
      const float* src = om.part + (int64_t)gm * N + n;
      float v = bias ? bias[n] : 0.f;
      for (int z = 0; z < S; ++z) v += __builtin_nontemporal_load(src + z * MN);
      if (relu) v = fmaxf(v, 0.f);
      const int64_t img = gm / om.rpi, rr = gm - img * om.rpi;
      if (n < om.split) Y[img * om.img_stride + rr * ldy + n] = (bf16)v;
      else om.Y2[img * om.img_stride2 + rr * om.ldy2 + (n - om.split)] = (bf16)v;
    }
    return;
  }
  // epilogue: bias + act, the bf16 tile staged in LDS (16-B chunks XOR-swizzled by row), then
  // written back as whole row segments, 16 B per lane (the direct 8-B-per-lane stores of 16-row
  // x 32-B fragments measured 1.4-1.9 TB/s on these write-heavy layers)
  constexpr int CH = BN / 8;  // 16-B chunks per tile row
  bf16* const sC = smem;      // [GBM][BN]; the loop's last barrier freed the operand ring
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn * WN + j * 16 + 4 * (lane >> 4);  // local column of this lane's 4 values
    const int gn = n0 + cl;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = (gn + r < N && bias) ? bias[gn + r] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wm * 64 + i * 16 + (lane & 15);
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = acc[i][j][r] + bv[r];
        o[r] = (bf16)(relu ? fmaxf(v, 0.f) : v);
      }
      *(bf16x4*)(sC + row * BN + (((cl >> 3) ^ (row & (CH - 1))) << 3) + (cl & 4)) = o;
    }
  }
  __syncthreads();
  for (int e = tid; e < GBM * CH; e += 256) {
    const int row = e / CH, ch = e - row * CH;
    const int gm = m0 + row, gn = n0 + ch * 8;
    if (gm >= M || gn >= N) continue;
    const bf16x8 v = *(const bf16x8*)(sC + row * BN + ((ch ^ (row & (CH - 1))) << 3));
    const int64_t img = gm / om.rpi, rr = gm - img * om.rpi;
    bf16* const lo = Y + img * om.img_stride + rr * ldy + gn;
    if (gn + 8 <= om.split && ((uintptr_t)lo & 15) == 0) {
      *(bf16x8*)lo = v;
      continue;
    }
    bf16* const hi = om.Y2 + img * om.img_stride2 + rr * om.ldy2 + (gn - om.split);
    if (gn >= om.split && gn + 8 <= N && ((uintptr_t)hi & 15) == 0) {
      *(bf16x8*)hi = v;
      continue;
    }
#pragma unroll
    for (int r = 0; r < 8; ++r) {
      const int n = gn + r;
      if (n >= N) break;
      if (n < om.split) Y[img * om.img_stride + rr * ldy + n] = v[r];
      else om.Y2[img * om.img_stride2 + rr * om.ldy2 + (n - om.split)] = v[r];
    }
  }
}

// =====================================================================================
// K5+K6 fused, 2-D pixel tiles: one workgroup = a TH x TW tile of output pixels of one image.
//   1. the input halo ((TH-1)S+3 x (TW-1)S+3 pixels x K channels) -> LDS, 16-B buffer loads
//      (rows above/below the image read as zero through the buffer range, side pad columns masked)
//   2. depthwise 3x3 + bias (+ReLU) from LDS (dot2 reduction, weights in registers) -> the
//      bf16 A tile [TH*TW px][K] in LDS (rounded where the two-kernel path rounds it)
//   3. pointwise GEMM on MFMA against W [N][K] (in LDS), + bias (+ReLU) -> staged in LDS ->
//      coalesced NHWC row segments.
// The depthwise activation never goes through HBM, and every input pixel is read from HBM once
// (plus the halo rows/columns neighbouring tiles share through L2). For the early, wide MobileNet
// blocks (conv1..conv3: 150^2 / 75^2 pixels, K = 32..128, N = 64..128). The 1-D-tile fusion
// inside the GEMM's A staging (AM_DW) re-read every tap from L1 (9x) and lost to two kernels.
// =====================================================================================
template <int K, int N, int S, int TH, int TW>
__global__ void __launch_bounds__(256) dwpw_tile_kernel(const bf16* __restrict__ x, const uint32_t* __restrict__ dwp,
                                                         const float* __restrict__ dwb, int dw_relu,
                                                         const bf16* __restrict__ Wt, const float* __restrict__ pb,
                                                         int relu, bf16* __restrict__ y, int H, int W, int Ho, int Wo) {
  constexpr int HH = (TH - 1) * S + 3, HW = (TW - 1) * S + 3;  // halo rows / columns
  constexpr int K8 = K / 8, MT = TH * TW, KS = K / 32;            // 8-ch groups, tile pixels, K slices
  constexpr int HALO_B = HH * HW * K * 2, A_B = MT * K * 2, W_B = N * K * 2, OUT_B = MT * N * 2;
  constexpr int R0 = HALO_B > OUT_B ? HALO_B : OUT_B;             // halo, later the output staging
  static_assert(256 % K8 == 0 && K % 32 == 0 && N % 64 == 0 && MT % 16 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[R0 + A_B + W_B];
  char* const halo = smem;
  bf16* const sA = (bf16*)(smem + R0);      // KS slices of [MT][32], gidx-swizzled
  bf16* const sW = (bf16*)(smem + R0 + A_B);  // KS slices of [N][32], gidx-swizzled
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int n = blockIdx.z, oy0 = blockIdx.y * TH, ox0 = blockIdx.x * TW;
  const int iy0 = oy0 * S - 1, ix0 = ox0 * S - 1;

  // ---- 1. halo + pointwise weights -> LDS
  const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)n * H * W * K), (short)0, H * W * K * 2,
                                                    0x00020000);
  for (int e = tid; e < HH * HW * K8; e += 256) {
    const int c = e % K8, px = e / K8, hx = px % HW, hy = px / HW;
    const int iy = iy0 + hy, ix = ix0 + hx;
    const int off = (ix >= 0 && ix < W) ? ((iy * W + ix) * K + c * 8) * 2 : (int)0x80000000;
    *(u32x4*)(halo + e * 16) = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
  for (int e = tid; e < N * K8; e += 256) {
    const int row = e / K8, c = e % K8;
    *(u32x4*)(sW + (c >> 2) * N * 32 + gidx(row, c & 3)) = *(const u32x4*)(Wt + (int64_t)row * K + c * 8);
  }
  // depthwise weights of this thread's channel group (fixed: 256 % K8 == 0), in registers
  const int c8 = tid % K8;
  uint32_t wr[5][8];
  load_dw_weights(dwp + c8 * 8, K, wr);
  const f32x4 db0 = *(const f32x4*)(dwb + c8 * 8), db1 = *(const f32x4*)(dwb + c8 * 8 + 4);
  __syncthreads();

  // ---- 2. depthwise from LDS -> A tile
  for (int p = tid / K8; p < MT; p += 256 / K8) {
    const int ty = p / TW, tx = p % TW;
    u32x4 t9[9];
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int hy = ty * S + t / 3, hx = tx * S + t % 3;
      t9[t] = *(const u32x4*)(halo + ((hy * HW + hx) * K + c8 * 8) * 2);
    }
    float a[8] = {db0[0], db0[1], db0[2], db0[3], db1[0], db1[1], db1[2], db1[3]};
    dw9_accum_w(t9, wr, a);
    *(u32x4*)(sA + (c8 >> 2) * MT * 32 + gidx(p, c8 & 3)) = dw_out8(a, dw_relu);
  }
  __syncthreads();

  // ---- 3. pointwise GEMM: wave w takes columns [w N/4, (w+1) N/4) for all MT rows
  constexpr int NB = N / 64, MB = MT / 16;
  f32x4 acc[MB][NB];
#pragma unroll
  for (int i = 0; i < MB; ++i)
#pragma unroll
    for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fc = lane >> 4;
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) {
    bf16x8s bw[NB];
#pragma unroll
    for (int j = 0; j < NB; ++j) bw[j] = *(const bf16x8s*)(sW + ks * N * 32 + gidx(wid * (N / 4) + j * 16 + fr, fc));
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const bf16x8s af = *(const bf16x8s*)(sA + ks * MT * 32 + gidx(i * 16 + fr, fc));
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af, acc[i][j], 0, 0, 0);
    }
  }
  // epilogue: acc[i][j][r] = out[px = 16 i + fr][col = w N/4 + 16 j + 4 fc + r], staged as [MT][N]
  // bf16 rows (16-B chunks XOR-swizzled by px) in the halo region (free since the barrier)
  bf16* const sO = (bf16*)halo;
  constexpr int CH = N / 8;
#pragma unroll
  for (int j = 0; j < NB; ++j) {
    const int col = wid * (N / 4) + j * 16 + 4 * fc;
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = pb[col + r];
#pragma unroll
    for (int i = 0; i < MB; ++i) {
      const int px = i * 16 + fr;
      bf16x4 o;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float v = acc[i][j][r] + bv[r];
        o[r] = (bf16)(relu ? fmaxf(v, 0.f) : v);
      }
      *(bf16x4*)(sO + px * N + (((col >> 3) ^ (px & (CH - 1))) << 3) + (col & 4)) = o;
    }
  }
  __syncthreads();
  for (int e = tid; e < MT * CH; e += 256) {
    const int px = e / CH, ch = e % CH, oy = oy0 + px / TW, ox = ox0 + px % TW;
    if (oy >= Ho || ox >= Wo) continue;
    *(u32x4*)(y + (((int64_t)n * Ho + oy) * Wo + ox) * N + ch * 8) =
        *(const u32x4*)(sO + px * N + ((ch ^ (px & (CH - 1))) << 3));
  }
}

// Persistent form of dwpw_tile_kernel: a workgroup walks tiles blockIdx.x, + gridDim.x, ... with
// the pointwise weights loaded into LDS ONCE (32 KB per tile launch at conv3: 300 MB of L2 reads
// over a chunk in the one-tile form) and the NEXT tile's halo loaded into registers while this
// tile's depthwise output goes through the MFMA GEMM and the stores, so the halo latency overlaps
// compute inside a workgroup, not only across the 2 co-resident workgroups of the conv2/conv3 forms.
template <int K, int N, int S, int TH, int TW>
__global__ void __launch_bounds__(256) dwpw_persist_kernel(const bf16* __restrict__ x, const uint32_t* __restrict__ dwp,
                                                            const float* __restrict__ dwb, int dw_relu,
                                                            const bf16* __restrict__ Wt, const float* __restrict__ pb,
                                                            int relu, bf16* __restrict__ y, int H, int W, int Ho, int Wo,
                                                            int imgs) {
  constexpr int HH = (TH - 1) * S + 3, HW = (TW - 1) * S + 3;
  constexpr int K8 = K / 8, MT = TH * TW, KS = K / 32;
  constexpr int HALO_B = HH * HW * K * 2, A_B = MT * K * 2, W_B = N * K * 2, OUT_B = MT * N * 2;
  constexpr int R0 = HALO_B > OUT_B ? HALO_B : OUT_B;
  constexpr int NE = HH * HW * K8, NH = (NE + 255) / 256;  // halo 16-B pieces, per thread
  static_assert(256 % K8 == 0 && K % 32 == 0 && N % 64 == 0 && MT % 16 == 0, "tile shape");
  __shared__ __attribute__((aligned(16))) char smem[R0 + A_B + W_B];
  char* const halo = smem;
  bf16* const sA = (bf16*)(smem + R0);
  bf16* const sW = (bf16*)(smem + R0 + A_B);
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int ntx = (Wo + TW - 1) / TW, nty = (Ho + TH - 1) / TH, per = ntx * nty, ntiles = per * imgs;
  for (int e = tid; e < N * K8; e += 256) {
    const int row = e / K8, c = e % K8;
    *(u32x4*)(sW + (c >> 2) * N * 32 + gidx(row, c & 3)) = *(const u32x4*)(Wt + (int64_t)row * K + c * 8);
  }
  const int c8 = tid % K8;
  uint32_t wr[5][8];
  load_dw_weights(dwp + c8 * 8, K, wr);
  const f32x4 db0 = *(const f32x4*)(dwb + c8 * 8), db1 = *(const f32x4*)(dwb + c8 * 8 + 4);
  u32x4 hr[NH];
  auto gload = [&](int t) {
    const int n = t / per, r = t - n * per;
    const int iy0 = (r / ntx) * TH * S - 1, ix0 = (r % ntx) * TW * S - 1;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)n * H * W * K), (short)0, H * W * K * 2,
                                                      0x00020000);
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const int e = tid + i * 256;
      if (e < NE) {
        const int c = e % K8, px = e / K8, hx = px % HW, hy = px / HW;
        const int iy = iy0 + hy, ix = ix0 + hx;
        const int off = (ix >= 0 && ix < W) ? ((iy * W + ix) * K + c * 8) * 2 : (int)0x80000000;
        hr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
  };
  if ((int)blockIdx.x < ntiles) gload(blockIdx.x);
  constexpr int NB = N / 64, MB = MT / 16, CH = N / 8;
  const int fr = lane & 15, fc = lane >> 4;
  bf16* const sO = (bf16*)halo;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / per, r = t - n * per, oy0 = (r / ntx) * TH, ox0 = (r % ntx) * TW;
    // 1. this tile's halo (registers) -> LDS (the previous tile's output staging there was drained
    //    before the barrier that ended the previous iteration)
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const int e = tid + i * 256;
      if (e < NE) *(u32x4*)(halo + e * 16) = hr[i];
    }
    __syncthreads();
    // 2. depthwise from LDS -> A tile
    for (int p = tid / K8; p < MT; p += 256 / K8) {
      const int ty = p / TW, tx = p % TW;
      u32x4 t9[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) {
        const int hy = ty * S + q / 3, hx = tx * S + q % 3;
        t9[q] = *(const u32x4*)(halo + ((hy * HW + hx) * K + c8 * 8) * 2);
      }
      float a[8] = {db0[0], db0[1], db0[2], db0[3], db1[0], db1[1], db1[2], db1[3]};
      dw9_accum_w(t9, wr, a);
      *(u32x4*)(sA + (c8 >> 2) * MT * 32 + gidx(p, c8 & 3)) = dw_out8(a, dw_relu);
    }
    __syncthreads();
    // 3. the next tile's halo loads go out now and land during the GEMM and the stores
    if (t + (int)gridDim.x < ntiles) gload(t + gridDim.x);
    // 4. pointwise GEMM (wave w: columns [w N/4, (w+1) N/4)), output staged in the halo region
    f32x4 acc[MB][NB];
#pragma unroll
    for (int i = 0; i < MB; ++i)
#pragma unroll
      for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      bf16x8s bw[NB];
#pragma unroll
      for (int j = 0; j < NB; ++j) bw[j] = *(const bf16x8s*)(sW + ks * N * 32 + gidx(wid * (N / 4) + j * 16 + fr, fc));
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const bf16x8s af = *(const bf16x8s*)(sA + ks * MT * 32 + gidx(i * 16 + fr, fc));
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af, acc[i][j], 0, 0, 0);
      }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int col = wid * (N / 4) + j * 16 + 4 * fc;
      float bv[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) bv[q] = pb[col + q];
#pragma unroll
      for (int i = 0; i < MB; ++i) {
        const int px = i * 16 + fr;
        bf16x4 o;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = acc[i][j][q] + bv[q];
          o[q] = (bf16)(relu ? fmaxf(v, 0.f) : v);
        }
        *(bf16x4*)(sO + px * N + (((col >> 3) ^ (px & (CH - 1))) << 3) + (col & 4)) = o;
      }
    }
    __syncthreads();
    // 5. coalesced NHWC row segments
    for (int e = tid; e < MT * CH; e += 256) {
      const int px = e / CH, ch = e % CH, oy = oy0 + px / TW, ox = ox0 + px % TW;
      if (oy >= Ho || ox >= Wo) continue;
      *(u32x4*)(y + (((int64_t)n * Ho + oy) * Wo + ox) * N + ch * 8) =
          *(const u32x4*)(sO + px * N + ((ch ^ (px & (CH - 1))) << 3));
    }
    __syncthreads();
  }
}

// =====================================================================================
// Two MobileNet blocks in one persistent kernel: conv1 (depthwise 3x3 s1 + pointwise K1 -> N1) and
// conv2 (depthwise 3x3 s2 + pointwise N1 -> N2), prototxt conv1/dw .. conv2 (MobileNetSSD_deploy:42-106).
// Unfused, conv1's output (150^2 x 64 bf16 = 288 MB per 100-frame chunk) is written by one kernel and
// read back by the next: 2 x 288 MB of the 864 MB the two blocks moved (216 us of the 1.19 ms chunk,
// profiles/r3_detector_chunk_final.txt). Here a workgroup owns a TH x TW tile of conv2's OUTPUT and
// recomputes the conv1 region it needs, (2 TH + 1) x (2 TW + 1) pixels, from a (2 TH + 3) x (2 TW + 3)
// halo of conv0's output: conv1's output lives only in LDS.
//   R0: the conv0 halo [HH*HW][K1] -> (after dw1) conv1's output P1 [PH*PW][N1] -> (after dw2) the
//       output staging [TH*TW][N2];  R1: dw1's output (pw1's A tile) -> (after pw1) dw2's output
//       (pw2's A tile);  W1, W2: the pointwise weights, loaded once per workgroup.
// P1 pixels outside the image are written as ZERO (conv2's depthwise padding), not as pw1 of zeros.
// Every intermediate is rounded to bf16 where the unfused kernels store it, and the reductions run in
// the same order (dw9_accum_w, one MFMA chain per K slice), so the result equals the two-kernel path.
// The next tile's halo is loaded into registers while this tile's GEMMs and stores run.
template <int K1, int N1, int N2, int TH, int TW>
struct Dwpw2 {
  static constexpr int PH = 2 * TH + 1, PW = 2 * TW + 1, MP = PH * PW, MP16 = (MP + 15) / 16 * 16;
  static constexpr int HH = PH + 2, HW = PW + 2, MT = TH * TW;
  static constexpr int HALO_B = HH * HW * K1 * 2, P1_B = MP * N1 * 2, OUT_B = MT * N2 * 2;
  static constexpr int R0 = (HALO_B > P1_B ? (HALO_B > OUT_B ? HALO_B : OUT_B) : (P1_B > OUT_B ? P1_B : OUT_B));
  static constexpr int A1_B = MP16 * K1 * 2, A2_B = MT * N1 * 2, R1 = A1_B > A2_B ? A1_B : A2_B;
  static constexpr int W1_B = N1 * K1 * 2, W2_B = N2 * N1 * 2;
  // dw2's paired weights [5][N1] dwords, the fp32 biases dw2 [N1], pw1 [N1], pw2 [N2], dw1's weights [5][K1]
  static constexpr int C_B = 5 * N1 * 4 + (2 * N1 + N2) * 4 + 5 * K1 * 4;
  static constexpr int LDS = R0 + R1 + W1_B + W2_B + C_B;
  static constexpr int NE = HH * HW * (K1 / 8), NH = (NE + 255) / 256;  // halo 16-B pieces (per thread)
};

template <int K1, int N1, int N2, int TH, int TW, int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE)))
dwpw2_persist_kernel(const bf16* __restrict__ x, const uint32_t* __restrict__ dwp1, const float* __restrict__ dwb1,
                     int dw1_relu, const bf16* __restrict__ Wt1, const float* __restrict__ pb1, int relu1,
                     const uint32_t* __restrict__ dwp2, const float* __restrict__ dwb2, int dw2_relu,
                     const bf16* __restrict__ Wt2, const float* __restrict__ pb2, int relu2, bf16* __restrict__ y,
                     int H, int W, int Ho, int Wo, int imgs) {
  using G = Dwpw2<K1, N1, N2, TH, TW>;
  constexpr int PW = G::PW, MP = G::MP, MP16 = G::MP16, HW = G::HW, MT = G::MT, NE = G::NE, NH = G::NH;
  constexpr int K18 = K1 / 8, N18 = N1 / 8, KS1 = K1 / 32, KS2 = N1 / 32;
  static_assert(256 % K18 == 0 && 256 % N18 == 0 && K1 % 32 == 0 && N1 % 64 == 0 && N2 % 64 == 0 && MT % 16 == 0,
                "tile shape");
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const r0 = smem;
  bf16* const sP1 = (bf16*)smem;                                  // R0 after dw1
  bf16* const sO = (bf16*)smem;                                   // R0 after dw2
  bf16* const sA = (bf16*)(smem + G::R0);                         // R1: A1, later A2
  bf16* const sW1 = (bf16*)(smem + G::R0 + G::R1);
  bf16* const sW2 = (bf16*)(smem + G::R0 + G::R1 + G::W1_B);
  uint32_t* const sDw2 = (uint32_t*)(smem + G::R0 + G::R1 + G::W1_B + G::W2_B);  // [5][N1] paired dw2 weights
  float* const sB = (float*)(sDw2 + 5 * N1);  // dw2 bias [N1] | pw1 bias [N1] | pw2 bias [N2]
  uint32_t* const sDw1 = (uint32_t*)(sB + 2 * N1 + N2);  // [5][K1] paired dw1 weights
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  for (int e = tid; e < 5 * N1; e += 256) sDw2[e] = dwp2[e];
  for (int e = tid; e < 5 * K1; e += 256) sDw1[e] = dwp1[e];
  for (int e = tid; e < 2 * N1 + N2; e += 256) sB[e] = e < N1 ? dwb2[e] : (e < 2 * N1 ? pb1[e - N1] : pb2[e - 2 * N1]);
  const int ntx = (Wo + TW - 1) / TW, nty = (Ho + TH - 1) / TH, per = ntx * nty, ntiles = per * imgs;
  for (int e = tid; e < N1 * K18; e += 256) {
    const int row = e / K18, c = e % K18;
    *(u32x4*)(sW1 + (c >> 2) * N1 * 32 + gidx(row, c & 3)) = *(const u32x4*)(Wt1 + (int64_t)row * K1 + c * 8);
  }
  for (int e = tid; e < N2 * N18; e += 256) {
    const int row = e / N18, c = e % N18;
    *(u32x4*)(sW2 + (c >> 2) * N2 * 32 + gidx(row, c & 3)) = *(const u32x4*)(Wt2 + (int64_t)row * N1 + c * 8);
  }
  const int c8a = tid % K18, c8b = tid % N18;  // this thread's channel groups in dw1 / dw2
  // both depthwise weight sets and the biases live in LDS and are read per tile phase (holding them in
  // registers spilled at 2-3 workgroups per CU)
  u32x4 hr[NH];
  // halo of tile t: conv0 rows 2 Y0 - 2 .. 2 Y0 + 2 TH, columns 2 X0 - 2 .. 2 X0 + 2 TW (zero outside)
  auto gload = [&](int t) {
    const int n = t / per, r = t - n * per;
    const int iy0 = (r / ntx) * TH * 2 - 2, ix0 = (r % ntx) * TW * 2 - 2;
    const auto rs = __builtin_amdgcn_make_buffer_rsrc((void*)(x + (int64_t)n * H * W * K1), (short)0, H * W * K1 * 2,
                                                      0x00020000);
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const int e = tid + i * 256;
      if (e < NE) {
        const int c = e % K18, px = e / K18, hx = px % HW, hy = px / HW;
        const int iy = iy0 + hy, ix = ix0 + hx;
        const int off = (iy >= 0 && iy < H && ix >= 0 && ix < W) ? ((iy * W + ix) * K1 + c * 8) * 2 : (int)0x80000000;
        hr[i] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
  };
  if ((int)blockIdx.x < ntiles) gload(blockIdx.x);
  const int fr = lane & 15, fc = lane >> 4;
  for (int t = blockIdx.x; t < ntiles; t += gridDim.x) {
    const int n = t / per, r = t - n * per, oy0 = (r / ntx) * TH, ox0 = (r % ntx) * TW;
    // 1. halo (registers) -> R0
#pragma unroll
    for (int i = 0; i < NH; ++i) {
      const int e = tid + i * 256;
      if (e < NE) *(u32x4*)(r0 + e * 16) = hr[i];
    }
    __syncthreads();
    // 2. dw1 over the conv1 region (PH x PW pixels) -> A1 (KS1 slices of [MP16][32])
    uint32_t wr1[5][8];
    load_dw_weights(sDw1 + c8a * 8, K1, wr1);
#pragma unroll 1
    for (int p = tid / K18; p < MP; p += 256 / K18) {
      const int py = p / PW, px = p % PW;
      u32x4 t9[9];
#pragma unroll
      for (int q = 0; q < 9; ++q) t9[q] = *(const u32x4*)(r0 + (((py + q / 3) * HW + px + q % 3) * K1 + c8a * 8) * 2);
      const f32x4 d1a = *(const f32x4*)(dwb1 + c8a * 8), d1b = *(const f32x4*)(dwb1 + c8a * 8 + 4);  // L1 hits
      float a[8] = {d1a[0], d1a[1], d1a[2], d1a[3], d1b[0], d1b[1], d1b[2], d1b[3]};
      dw9_accum_w(t9, wr1, a);
      *(u32x4*)(sA + (c8a >> 2) * MP16 * 32 + gidx(p, c8a & 3)) = dw_out8(a, dw1_relu);
    }
    __syncthreads();
    // 3. pw1: wave w takes columns [w N1/4, (w+1) N1/4) of all MP16 rows, in two row passes (fewer live
    //    accumulators: the kernel runs at 2 workgroups per CU); results -> P1 in R0 as [MP][N1] bf16
    //    (+ bias, ReLU), pixels outside the image as 0
    {
      constexpr int NB = N1 / 64, MB = MP16 / 16, MBH = (MB + 1) / 2;
      const int r1 = oy0 * 2 - 1, c1 = ox0 * 2 - 1;  // conv1 coordinates of P1's pixel (0, 0)
#pragma unroll 1
      for (int half = 0; half < 2; ++half) {
        f32x4 acc[MBH][NB];
#pragma unroll
        for (int i = 0; i < MBH; ++i)
#pragma unroll
          for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int ks = 0; ks < KS1; ++ks) {
          bf16x8s bw[NB];
#pragma unroll
          for (int j = 0; j < NB; ++j) bw[j] = *(const bf16x8s*)(sW1 + ks * N1 * 32 + gidx(wid * (N1 / 4) + j * 16 + fr, fc));
#pragma unroll
          for (int i = 0; i < MBH; ++i) {
            const int ib = half * MBH + i;
            if (ib >= MB) continue;
            const bf16x8s af = *(const bf16x8s*)(sA + ks * MP16 * 32 + gidx(ib * 16 + fr, fc));
#pragma unroll
            for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af, acc[i][j], 0, 0, 0);
          }
        }
#pragma unroll
        for (int j = 0; j < NB; ++j) {
          const int col = wid * (N1 / 4) + j * 16 + 4 * fc;
          float bv[4];
#pragma unroll
          for (int q = 0; q < 4; ++q) bv[q] = sB[N1 + col + q];
#pragma unroll
          for (int i = 0; i < MBH; ++i) {
            const int px = (half * MBH + i) * 16 + fr;
            if (px >= MP) continue;
            const int yy = r1 + px / PW, xx = c1 + px % PW;
            const bool in = yy >= 0 && yy < H && xx >= 0 && xx < W;
            bf16x4 o;
#pragma unroll
            for (int q = 0; q < 4; ++q) {
              const float v = acc[i][j][q] + bv[q];
              o[q] = (bf16)(in ? (relu1 ? fmaxf(v, 0.f) : v) : 0.f);
            }
            // P1 rows are 128 B: the 16-B chunk index is XOR-swizzled by the pixel (else the 16 rows of an
            // MFMA block land on the same banks)
            *(bf16x4*)(sP1 + px * N1 + (((col >> 3) ^ (px & 7)) << 3) + (col & 4)) = o;
          }
        }
      }
    }
    // 4. the next tile's halo loads go out now (R0's halo is dead since dw1) and land during the rest
    if (t + (int)gridDim.x < ntiles) gload(t + gridDim.x);
    __syncthreads();
    // 5. dw2 (stride 2) from P1 -> A2 (KS2 slices of [MT][32]) in R1 (A1 is dead)
    uint32_t wr2[5][8];
    load_dw_weights(sDw2 + c8b * 8, N1, wr2);
    const f32x4 d2a = *(const f32x4*)(sB + c8b * 8), d2b = *(const f32x4*)(sB + c8b * 8 + 4);
#pragma unroll 1
    for (int q = tid / N18; q < MT; q += 256 / N18) {
      const int ty = q / TW, tx = q % TW;
      u32x4 t9[9];
#pragma unroll
      for (int u = 0; u < 9; ++u) {
        const int pp = (2 * ty + u / 3) * PW + 2 * tx + u % 3;
        t9[u] = *(const u32x4*)(sP1 + pp * N1 + ((c8b ^ (pp & 7)) << 3));
      }
      float a[8] = {d2a[0], d2a[1], d2a[2], d2a[3], d2b[0], d2b[1], d2b[2], d2b[3]};
      dw9_accum_w(t9, wr2, a);
      *(u32x4*)(sA + (c8b >> 2) * MT * 32 + gidx(q, c8b & 3)) = dw_out8(a, dw2_relu);
    }
    __syncthreads();
    // 6. pw2: wave w takes columns [w N2/4, (w+1) N2/4); output staged in R0 (P1 is dead)
    {
      constexpr int NB = N2 / 64, MB = MT / 16, CH = N2 / 8;
      f32x4 acc[MB][NB];
#pragma unroll
      for (int i = 0; i < MB; ++i)
#pragma unroll
        for (int j = 0; j < NB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int ks = 0; ks < KS2; ++ks) {
        bf16x8s bw[NB];
#pragma unroll
        for (int j = 0; j < NB; ++j) bw[j] = *(const bf16x8s*)(sW2 + ks * N2 * 32 + gidx(wid * (N2 / 4) + j * 16 + fr, fc));
#pragma unroll
        for (int i = 0; i < MB; ++i) {
          const bf16x8s af = *(const bf16x8s*)(sA + ks * MT * 32 + gidx(i * 16 + fr, fc));
#pragma unroll
          for (int j = 0; j < NB; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bw[j], af, acc[i][j], 0, 0, 0);
        }
      }
#pragma unroll
      for (int j = 0; j < NB; ++j) {
        const int col = wid * (N2 / 4) + j * 16 + 4 * fc;
        float bv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) bv[q] = sB[2 * N1 + col + q];
#pragma unroll
        for (int i = 0; i < MB; ++i) {
          const int px = i * 16 + fr;
          bf16x4 o;
#pragma unroll
          for (int q = 0; q < 4; ++q) {
            const float v = acc[i][j][q] + bv[q];
            o[q] = (bf16)(relu2 ? fmaxf(v, 0.f) : v);
          }
          *(bf16x4*)(sO + px * N2 + (((col >> 3) ^ (px & (CH - 1))) << 3) + (col & 4)) = o;
        }
      }
      __syncthreads();
      // 7. coalesced NHWC row segments
      for (int e = tid; e < MT * CH; e += 256) {
        const int px = e / CH, ch = e % CH, oy = oy0 + px / TW, ox = ox0 + px % TW;
        if (oy >= Ho || ox >= Wo) continue;
        *(u32x4*)(y + (((int64_t)n * Ho + oy) * Wo + ox) * N2 + ch * 8) =
            *(const u32x4*)(sO + px * N2 + ((ch ^ (px & (CH - 1))) << 3));
      }
    }
    __syncthreads();
  }
}

// =====================================================================================
// K4: the stem, conv0 3x3 (stride 2, pad 1) over the 4-channel padded blob, as MFMA fed straight
// from global memory: with K = 9 taps x 4 channels the v_mfma_f32_16x16x32_bf16 operand a lane
// holds (8 consecutive k = two whole taps of one pixel) is exactly two 8-B loads, so neither an
// LDS tile nor an im2col exists; the weight fragments (Cout x 64 k) stay in registers for the
// wave's life. One wave = 64 output pixels (4 MFMA row groups) x COUT channels.
// (The generic implicit GEMM spent 119 us on this layer: 2 K-steps per 128-row tile, half of
// every 64-wide N tile idle.)
// =====================================================================================
template <int COUT>
__global__ void __launch_bounds__(256) stem_conv_c4_kernel(const bf16* __restrict__ x, const bf16* __restrict__ wt,
                                                            const float* __restrict__ bias, bf16* __restrict__ y,
                                                            int M, int H, int W, int Ho, int Wo, int stride, int pad,
                                                            int relu) {
  constexpr int NT = COUT / 16;
  typedef short sx4v __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63;
  const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int r = lane & 15, q = lane >> 4;
  // weight fragments: out channel 16 t + r, k = 32 s + 8 q .. + 7 (columns (ky, kx, c), Kp = 64)
  bf16x8s wf[NT][2];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int st = 0; st < 2; ++st) wf[t][st] = *(const bf16x8s*)(wt + (16 * t + r) * 64 + 32 * st + 8 * q);
  float bv[NT][4];
#pragma unroll
  for (int t = 0; t < NT; ++t)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[t][i] = bias[16 * t + 4 * q + i];
  const int hw = Ho * Wo;
  auto tap = [&](int img, int iy0, int ix0, int tp) -> sx4v {  // 4 channels of tap tp, or zeros
    if (tp >= 9) return sx4v{0, 0, 0, 0};
    const int iy = iy0 + tp / 3, ix = ix0 + tp % 3;
    if (iy < 0 || iy >= H || ix < 0 || ix >= W) return sx4v{0, 0, 0, 0};
    return *(const sx4v*)(x + (((int64_t)img * H + iy) * W + ix) * 4);
  };
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int m = wave * 64 + g * 16 + r;  // this lane's pixel in MFMA row group g
    const bool ok = m < M;
    const int mm = ok ? m : M - 1;
    const int img = mm / hw, rem = mm - img * hw, oy = rem / Wo, ox = rem - oy * Wo;
    const int iy0 = oy * stride - pad, ix0 = ox * stride - pad;
    // k chunk q of step 0: taps 2q, 2q+1; of step 1: taps 8 + 2q, 9 + 2q (only tap 8 is real)
    const sx4v a0 = tap(img, iy0, ix0, 2 * q), a1 = tap(img, iy0, ix0, 2 * q + 1);
    const sx4v b0 = tap(img, iy0, ix0, 8 + 2 * q);
    const bf16x8s x0 = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    const bf16x8s x1 = {b0[0], b0[1], b0[2], b0[3], 0, 0, 0, 0};
#pragma unroll
    for (int t = 0; t < NT; ++t) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][0], x0, acc, 0, 0, 0);
      acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][1], x1, acc, 0, 0, 0);
      // acc[i] = out channel 16 t + 4 q + i of pixel m
      bf16x4 o;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float v = acc[i] + bv[t][i];
        o[i] = (bf16)(relu ? fmaxf(v, 0.f) : v);
      }
      if (ok) *(bf16x4*)(y + (int64_t)m * COUT + 16 * t + 4 * q) = o;
    }
  }
}

// =====================================================================================
// K12+K13: DetectionOutput. Stage 1: one block per (image, foreground class).
//   softmax(conf row)[class] > thresh -> candidates -> bitonic sort (desc score, asc prior)
//   -> top_k -> CENTER_SIZE decode -> greedy NMS -> per-class kept list.
// conf: [N, P, C] bf16 raw logits (the softmax is fused here), loc: [N, P, 4] bf16,
// pri: [P*4] fp32 boxes, var: [P*4] fp32.
// cls_out: [N, C, TOPK, 5] fp32 (score, x0, y0, x1, y1), cls_cnt: [N, C] int.
// =====================================================================================
constexpr int DET_MAXP = 2048;

// Stage 0: the per-prior class softmax (prototxt mbox_conf_softmax), ONCE per prior: one thread
// per (image, prior) reads its C logits and writes the C probabilities class-major,
// prob[n][c][p], so each class block of stage 1 streams one contiguous row (before: every one of
// the C-1 class blocks recomputed the whole C-way softmax of every prior).
__global__ void __launch_bounds__(256) ssd_softmax_kernel(const bf16* __restrict__ conf, float* __restrict__ prob,
                                                           int N, int P, int C) {
  const int64_t total = (int64_t)N * P;
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int n = (int)(i / P), p = (int)(i - (int64_t)n * P);
    const bf16* row = conf + i * C;
    float v[32];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k < C) {
        v[k] = (float)row[k];
        mx = fmaxf(mx, v[k]);
      }
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k < C) {
        v[k] = __expf(v[k] - mx);
        sum += v[k];
      }
    const float inv = 1.f / sum;
    float* o = prob + (int64_t)n * C * P + p;
#pragma unroll
    for (int k = 0; k < 32; ++k)
      if (k < C) o[(int64_t)k * P] = v[k] * inv;
  }
}

__global__ void __launch_bounds__(256) ssd_class_nms_kernel(const float* __restrict__ prob, const bf16* __restrict__ loc,
                                                             const float* __restrict__ pri, const float* __restrict__ var,
                                                             float* __restrict__ cls_out, int* __restrict__ cls_cnt,
                                                             int P, int C, int bg, float thresh, float nms_thresh,
                                                             int topk) {
  __shared__ float s_score[DET_MAXP];
  __shared__ int s_idx[DET_MAXP];
  __shared__ float s_box[DET_MAXP / 8][4];  // topk <= 256
  __shared__ int s_keep[DET_MAXP / 8];
  __shared__ int s_cnt;
  const int n = blockIdx.x / (C - 1);
  int c = blockIdx.x % (C - 1);
  c = c >= bg ? c + 1 : c;
  const int tid = threadIdx.x;
  if (tid == 0) s_cnt = 0;
  __syncthreads();
  const float* pr = prob + ((int64_t)n * C + c) * P;
  for (int p = tid; p < P; p += 256) {
    const float pv = pr[p];
    if (pv > thresh) {
      const int slot = atomicAdd(&s_cnt, 1);
      s_score[slot] = pv;
      s_idx[slot] = p;
    }
  }
  __syncthreads();
  const int ncand = s_cnt;
  int L = 1;
  while (L < ncand) L <<= 1;
  for (int i = ncand + tid; i < L; i += 256) {
    s_score[i] = -INFINITY;
    s_idx[i] = 0x7fffffff;
  }
  __syncthreads();
  // bitonic sort, descending by score, ascending by prior index on ties
  for (int k = 2; k <= L; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < L; i += 256) {
        const int ij = i ^ j;
        if (ij > i) {
          const bool desc = (i & k) == 0;
          const float a = s_score[i], b = s_score[ij];
          const int ia = s_idx[i], ib = s_idx[ij];
          const bool a_first = (a > b) || (a == b && ia < ib);
          if (desc ? !a_first : a_first) {
            s_score[i] = b;
            s_score[ij] = a;
            s_idx[i] = ib;
            s_idx[ij] = ia;
          }
        }
      }
      __syncthreads();
    }
  }
  const int K = min(ncand, topk);
  const bf16* lr = loc + (int64_t)n * P * 4;
  for (int i = tid; i < K; i += 256) {
    const int p = s_idx[i];
    const float px0 = pri[p * 4], py0 = pri[p * 4 + 1], px1 = pri[p * 4 + 2], py1 = pri[p * 4 + 3];
    const float pw = px1 - px0, ph = py1 - py0, pcx = 0.5f * (px0 + px1), pcy = 0.5f * (py0 + py1);
    const float cx = var[p * 4] * (float)lr[p * 4] * pw + pcx;
    const float cy = var[p * 4 + 1] * (float)lr[p * 4 + 1] * ph + pcy;
    const float bw = __expf(var[p * 4 + 2] * (float)lr[p * 4 + 2]) * pw;
    const float bh = __expf(var[p * 4 + 3] * (float)lr[p * 4 + 3]) * ph;
    s_box[i][0] = cx - 0.5f * bw;
    s_box[i][1] = cy - 0.5f * bh;
    s_box[i][2] = cx + 0.5f * bw;
    s_box[i][3] = cy + 0.5f * bh;
    s_keep[i] = 1;
  }
  __syncthreads();
  // greedy NMS: candidate i survives if no earlier survivor overlaps it by > nms_thresh
  for (int i = 0; i < K; ++i) {
    if (s_keep[i]) {
      const float ax0 = s_box[i][0], ay0 = s_box[i][1], ax1 = s_box[i][2], ay1 = s_box[i][3];
      const float aa = fmaxf(ax1 - ax0, 0.f) * fmaxf(ay1 - ay0, 0.f);
      for (int j = i + 1 + tid; j < K; j += 256) {
        if (!s_keep[j]) continue;
        const float bx0 = s_box[j][0], by0 = s_box[j][1], bx1 = s_box[j][2], by1 = s_box[j][3];
        const float iw = fminf(ax1, bx1) - fmaxf(ax0, bx0), ih = fminf(ay1, by1) - fmaxf(ay0, by0);
        const float inter = fmaxf(iw, 0.f) * fmaxf(ih, 0.f);
        const float ba = fmaxf(bx1 - bx0, 0.f) * fmaxf(by1 - by0, 0.f);
        const float uni = aa + ba - inter;
        const float iou = uni > 0.f ? inter / uni : 0.f;
        if (iou > nms_thresh) s_keep[j] = 0;
      }
    }
    __syncthreads();
  }
  if (tid == 0) {
    int w = 0;
    float* o = cls_out + ((int64_t)n * C + c) * topk * 5;
    for (int i = 0; i < K; ++i) {
      if (!s_keep[i]) continue;
      o[w * 5 + 0] = s_score[i];
      o[w * 5 + 1] = s_box[i][0];
      o[w * 5 + 2] = s_box[i][1];
      o[w * 5 + 3] = s_box[i][2];
      o[w * 5 + 4] = s_box[i][3];
      ++w;
    }
    cls_cnt[n * C + c] = w;
  }
}

// Stage 2: one block per image. Concatenate the per-class lists (class-major, as Caffe does);
// if more than keep_top_k survive, keep the keep_top_k highest scores (sorted descending).
// out: [N, KEEP, 7] (img, label, score, x0, y0, x1, y1), out_cnt: [N]
__global__ void __launch_bounds__(256) ssd_merge_kernel(const float* __restrict__ cls_out,
                                                         const int* __restrict__ cls_cnt, float* __restrict__ out,
                                                         int* __restrict__ out_cnt, int C, int bg, int topk, int keep) {
  __shared__ float s_score[DET_MAXP * 2];
  __shared__ int s_key[DET_MAXP * 2];  // class * topk + slot
  __shared__ int s_off[64];
  const int n = blockIdx.x, tid = threadIdx.x;
  if (tid == 0) {
    int o = 0;
    for (int c = 0; c < C; ++c) {
      s_off[c] = o;
      if (c != bg) o += cls_cnt[n * C + c];
    }
    s_off[C] = o;
  }
  __syncthreads();
  const int total = s_off[C];
  const float* co = cls_out + (int64_t)n * C * topk * 5;
  float* on = out + (int64_t)n * keep * 7;
  if (total <= keep) {
    for (int c = 0; c < C; ++c) {
      if (c == bg) continue;
      const int cnt = cls_cnt[n * C + c];
      for (int s = tid; s < cnt; s += 256) {
        const float* src = co + ((int64_t)c * topk + s) * 5;
        float* d = on + (int64_t)(s_off[c] + s) * 7;
        d[0] = (float)n; d[1] = (float)c; d[2] = src[0];
        d[3] = src[1]; d[4] = src[2]; d[5] = src[3]; d[6] = src[4];
      }
    }
    for (int i = total * 7 + tid; i < keep * 7; i += 256) on[i] = 0.f;  // zero padding (out is not pre-zeroed)
    if (tid == 0) out_cnt[n] = total;
    return;
  }
  int L = 1;
  while (L < total) L <<= 1;
  for (int c = 0; c < C; ++c) {
    if (c == bg) continue;
    const int cnt = cls_cnt[n * C + c];
    for (int s = tid; s < cnt; s += 256) {
      s_score[s_off[c] + s] = co[((int64_t)c * topk + s) * 5];
      s_key[s_off[c] + s] = c * topk + s;
    }
  }
  for (int i = total + tid; i < L; i += 256) {
    s_score[i] = -INFINITY;
    s_key[i] = 0x7fffffff;
  }
  __syncthreads();
  for (int k = 2; k <= L; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = tid; i < L; i += 256) {
        const int ij = i ^ j;
        if (ij > i) {
          const bool desc = (i & k) == 0;
          const float a = s_score[i], b = s_score[ij];
          const int ka = s_key[i], kb = s_key[ij];
          const bool a_first = (a > b) || (a == b && ka < kb);
          if (desc ? !a_first : a_first) {
            s_score[i] = b; s_score[ij] = a;
            s_key[i] = kb; s_key[ij] = ka;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < keep; i += 256) {
    const int key = s_key[i], c = key / topk, s = key % topk;
    const float* src = co + ((int64_t)c * topk + s) * 5;
    float* d = on + (int64_t)i * 7;
    d[0] = (float)n; d[1] = (float)c; d[2] = src[0];
    d[3] = src[1]; d[4] = src[2]; d[5] = src[3]; d[6] = src[4];
  }
  if (tid == 0) out_cnt[n] = keep;
}

// =====================================================================================
// K14: annotation. One block per frame: 2-px boxes for `label` detections above `thresh`
// (colour box_bgr), then two pre-rasterised text masks: the requester name and the
// "person: k" label chosen by the per-frame count k (mask table indexed by k).
// frames: [N, h, w, 3] uint8 BGR (in place); dets: [N, KEEP, 7]; det_cnt: [N]
// =====================================================================================
__global__ void __launch_bounds__(256) annotate_kernel(uint8_t* __restrict__ frames, int h, int w,
                                                        const float* __restrict__ dets, const int* __restrict__ det_cnt,
                                                        int keep, int label, float thresh, uint32_t box_bgr,
                                                        const uint8_t* __restrict__ name_mask, int nm_h, int nm_w,
                                                        int nm_x, int nm_y, uint32_t name_bgr,
                                                        const uint8_t* __restrict__ lab_masks, int lm_n, int lm_h,
                                                        int lm_w, int lm_x, int lm_y, uint32_t lab_bgr,
                                                        int* __restrict__ counts_out) {
  __shared__ int s_count;
  const int n = blockIdx.x, tid = threadIdx.x;
  uint8_t* f = frames + (int64_t)n * h * w * 3;
  const float* dn = dets + (int64_t)n * keep * 7;
  const int nd = det_cnt[n];
  if (tid == 0) s_count = 0;
  __syncthreads();
  auto put = [&](int x, int y, uint32_t bgr) {
    if (x >= 0 && x < w && y >= 0 && y < h) {
      uint8_t* p = f + ((int64_t)y * w + x) * 3;
      p[0] = bgr & 255;
      p[1] = (bgr >> 8) & 255;
      p[2] = (bgr >> 16) & 255;
    }
  };
  for (int d = 0; d < nd; ++d) {
    const float* det = dn + d * 7;
    if ((int)det[1] != label || det[2] <= thresh) continue;
    if (tid == 0) s_count++;
    // box = det[3:7] * [w, h, w, h], truncated like ndarray.astype("int")
    const int x0 = (int)(det[3] * w), y0 = (int)(det[4] * h), x1 = (int)(det[5] * w), y1 = (int)(det[6] * h);
    const int bw = x1 - x0 + 1, bh = y1 - y0 + 1;
    if (bw <= 0 || bh <= 0 || bw > 4 * w || bh > 4 * h) continue;
    for (int t = tid; t < 2 * bw + 2 * bh; t += 256) {  // thickness 2: the line and its outer neighbour
      int x, y;
      if (t < bw) { x = x0 + t; y = y0; }
      else if (t < 2 * bw) { x = x0 + t - bw; y = y1; }
      else if (t < 2 * bw + bh) { x = x0; y = y0 + t - 2 * bw; }
      else { x = x1; y = y0 + t - 2 * bw - bh; }
      put(x, y, box_bgr);
      if (y == y0) put(x, y - 1, box_bgr);
      else if (y == y1) put(x, y + 1, box_bgr);
      if (x == x0) put(x - 1, y, box_bgr);
      else if (x == x1) put(x + 1, y, box_bgr);
    }
  }
  __syncthreads();
  for (int t = tid; t < nm_h * nm_w; t += 256) {
    if (name_mask[t]) put(nm_x + t % nm_w, nm_y + t / nm_w, name_bgr);
  }
  const int k = min(s_count, lm_n - 1);
  const uint8_t* lm = lab_masks + (int64_t)k * lm_h * lm_w;
  for (int t = tid; t < lm_h * lm_w; t += 256) {
    if (lm[t]) put(lm_x + t % lm_w, lm_y + t / lm_w, lab_bgr);
  }
  if (tid == 0 && counts_out) counts_out[n] = s_count;
}

}  // namespace vcx

// ====================================================================================== launchers
using namespace vcx;

void vcx_resize_area_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int h, int w, hipStream_t s) {
  const float sx = (float)W / w, sy = (float)H / h;
  const int taps = (int)ceilf(sx) + 1;  // input columns an output column can touch
  if ((W * 3) % 16 == 0 && ((uintptr_t)src & 15) == 0 && w <= RA_XMAX * 256 && W * 3 <= RA_LDS && h <= H &&
      w <= W && W >= 8 && taps <= 8 && (int64_t)N * h < INT32_MAX) {
    if (taps <= 5)
      hipLaunchKernelGGL(resize_area_rows_kernel<5>, dim3(N * h), dim3(256), 0, s, src, dst, N, H, W, h, w, sx, sy);
    else
      hipLaunchKernelGGL(resize_area_rows_kernel<8>, dim3(N * h), dim3(256), 0, s, src, dst, N, H, W, h, w, sx, sy);
    return;
  }
  hipLaunchKernelGGL(resize_area_u8_kernel, dim3(stream_grid((int64_t)N * h * w, 256)), dim3(256), 0, s, src, dst, N,
                     H, W, h, w);
}

void vcx_resize_bilinear_u8(const uint8_t* src, uint8_t* dst, int N, int H, int W, int h, int w, hipStream_t s) {
  hipLaunchKernelGGL(resize_bilinear_u8_kernel, dim3(stream_grid((int64_t)N * h * w, 256)), dim3(256), 0, s, src, dst,
                     N, H, W, h, w);
}

void vcx_blob_bilinear(const uint8_t* src, void* dst, int N, int H, int W, int S, float scale, float mean,
                       hipStream_t s) {
  const float sx = (float)W / S, sy = (float)H / S;
  constexpr int RB = 8;
  const int64_t rows_lds = ((int64_t)((RB - 1) * sy) + 3) * W * 3 + 1024;  // + the DMA tail's overrun
  static const bool rows_form = [] {
    const char* e = std::getenv("VCX_BLOB_ROWS");
    return !(e && e[0] == '0');
  }();
  if (rows_form && (W * 3) % 16 == 0 && rows_lds <= 48 * 1024 && ((uintptr_t)src & 15) == 0) {
    const int bt = std::min(320, (S + 63) / 64 * 64);
    hipLaunchKernelGGL(blob_bilinear_rows_kernel<RB>, dim3(1, (S + RB - 1) / RB, N), dim3(bt), (size_t)rows_lds, s, src,
                       (bf16*)dst, N, H, W, S, sx, sy, scale, mean);
    return;
  }
  if ((W * 3) % 16 == 0 && W * 3 <= BLOB_LDS && ((uintptr_t)src & 15) == 0) {
    const int bt = std::min(320, (S + 63) / 64 * 64);
    hipLaunchKernelGGL(blob_bilinear_kernel, dim3(1, S, N), dim3(bt), 0, s, src, (bf16*)dst, N, H, W, S, sx, sy, scale,
                       mean);
  } else {
    hipLaunchKernelGGL(blob_bilinear_any_kernel, dim3((S + 255) / 256, S, N), dim3(256), 0, s, src, (bf16*)dst, N, H,
                       W, S, sx, sy, scale, mean);
  }
}

void vcx_im2col_nhwc(const void* x, void* out, int N, int H, int W, int C, int Cs, int Ho, int Wo, int KH, int KW,
                     int stride, int pad, int Kp, hipStream_t s) {
  hipLaunchKernelGGL(im2col_nhwc_kernel, dim3(stream_grid((int64_t)N * Ho * Wo * Kp, 256)), dim3(256), 0, s,
                     (const bf16*)x, (bf16*)out, N, H, W, C, Cs, Ho, Wo, KH, KW, stride, pad, Kp);
}

void vcx_dwconv3x3(const void* x, const void* w, const float* b, void* y, int N, int H, int W, int C, int Ho, int Wo,
                   int stride, int relu, hipStream_t s) {
  int sh = 0;
  while ((8 << sh) < C) ++sh;
  if ((8 << sh) != C) sh = -1;  // C8 = C / 8 = 1 << sh, or -1: not a power of two
  const int bx = (Wo * (C / 8) + 255) / 256;
  if (stride == 1) {
    constexpr int R = 4;
    hipLaunchKernelGGL((dwconv3x3_kernel<1, R>), dim3(bx, N * ((Ho + R - 1) / R)), dim3(256), 0, s, (const bf16*)x,
                       (const uint32_t*)w, b, (bf16*)y, H, W, C, Ho, Wo, sh, relu);
  } else {
    constexpr int R = 2;
    hipLaunchKernelGGL((dwconv3x3_kernel<2, R>), dim3(bx, N * ((Ho + R - 1) / R)), dim3(256), 0, s, (const bf16*)x,
                       (const uint32_t*)w, b, (bf16*)y, H, W, C, Ho, Wo, sh, relu);
  }
}

// K-split factor for a launch that would leave most CUs idle (the SSD extras and heads: M = 100..
// 10,000 rows, K up to 2,304): each z-slice of the grid takes K / S columns, fp32 partials go to a
// workspace and splitk_bias_act applies bias/ReLU/mapping. 1 = no split.
int vcx_vision_ksplit(int M, int N, int K) {
  const int nwg = ((M + GBM - 1) / GBM) * ((N + (N <= 64 ? 63 : 127)) / (N <= 64 ? 64 : 128));
  if (nwg >= 192 || K < 256) return 1;
  int S = std::min(8, std::min(K / 128, (384 + nwg - 1) / nwg));
  while (S > 1 && (K / GBK) % S) --S;
  return std::max(S, 1);
}

template <int AM>
static void launch_gba(const bf16* X, const bf16* Wt, const float* bias, bf16* Y, int M, int N, int K, int ldy,
                       int relu, OutMap om, const ConvGeom& cg, float* ws, int S, int* cnt, hipStream_t s) {
  if (S > 1) {
    om.part = ws;
    om.kchunk = K / S;
    om.cnt = cnt;
  }
  const int tm = (M + GBM - 1) / GBM;
  if (N <= 64)
    hipLaunchKernelGGL((gemm_bias_act_kernel<64, AM>), dim3(tm * ((N + 63) / 64), 1, S), dim3(256), 0, s, X, Wt, bias,
                       Y, M, N, K, ldy, relu, om, cg);
  else
    hipLaunchKernelGGL((gemm_bias_act_kernel<128, AM>), dim3(tm * ((N + 127) / 128), 1, S), dim3(256), 0, s, X, Wt,
                       bias, Y, M, N, K, ldy, relu, om, cg);
  if (S > 1 && !cnt) {
    om.part = nullptr;
    hipLaunchKernelGGL(splitk_bias_act_kernel, dim3(stream_grid((int64_t)M * N, 256)), dim3(256), 0, s, ws, S, bias,
                       Y, M, N, ldy, relu, om);
  }
}

void vcx_gemm_bias_act_mapped(const void* X, const void* Wt, const float* bias, void* Y, int M, int N, int K, int ldy,
                              int relu, void* Y2, int split, int ldy2, int rpi, int64_t img_stride,
                              int64_t img_stride2, float* ws, int S, int* cnt, hipStream_t s) {
  OutMap om{(bf16*)Y2, split, ldy2, rpi > 0 ? rpi : M, img_stride, img_stride2, nullptr, 0, nullptr};
  ConvGeom cg{};
  launch_gba<AM_PLAIN>((const bf16*)X, (const bf16*)Wt, bias, (bf16*)Y, M, N, K, ldy, relu, om, cg, ws, S, cnt, s);
}

// Y [imgs*Ho*Wo, N] = act(conv(x) + bias): x NHWC [imgs, H, W, Cs] (C used channels), weights
// Wt [N, Kp] with columns (ky, kx, c), Kp % 32 == 0 (zero beyond KH*KW*C)
void vcx_conv_implicit(const void* x, const void* Wt, const float* bias, void* Y, int imgs, int H, int W, int C,
                       int Cs, int KH, int KW, int stride, int pad, int N, int Kp, int relu, float* ws, int S,
                       int* cnt, hipStream_t s) {
  const int Ho = (H + 2 * pad - KH) / stride + 1, Wo = (W + 2 * pad - KW) / stride + 1;
  const int M = imgs * Ho * Wo;
  if (C == 4 && Cs == 4 && KH == 3 && KW == 3 && Kp == 64 && (N == 16 || N == 32 || N == 64)) {
    const int blocks = (M + 255) / 256;  // 4 waves x 64 pixels
    auto go = [&](auto kern) {
      hipLaunchKernelGGL(kern, dim3(blocks), dim3(256), 0, s, (const bf16*)x, (const bf16*)Wt, bias, (bf16*)Y, M, H,
                         W, Ho, Wo, stride, pad, relu);
    };
    if (N == 16) go(stem_conv_c4_kernel<16>);
    else if (N == 32) go(stem_conv_c4_kernel<32>);
    else go(stem_conv_c4_kernel<64>);
    return;
  }
  OutMap om{nullptr, N, 0, M, 0, 0, nullptr, 0, nullptr};
  ConvGeom cg{H, W, C, Cs, Ho, Wo, KW, stride, pad, KH * KW * C, nullptr, nullptr, 0};
  launch_gba<AM_IMPLICIT>((const bf16*)x, (const bf16*)Wt, bias, (bf16*)Y, M, N, Kp, N, relu, om, cg, ws, S, cnt, s);
}

static int vision_cus() {
  static int n = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = 256;
    return c;
  }();
  return n;
}

// depthwise 3x3 (pad 1) + bias (+ReLU) -> pointwise GEMM + bias (+ReLU), one kernel:
// x NHWC [imgs, H, W, K], dw_w [5][K] paired, dw_b [K], Wt [N, K] -> Y [imgs*Ho*Wo, N]
void vcx_dw_pw(const void* x, const void* dw_w, const float* dw_b, int dw_relu, const void* Wt, const float* bias,
               void* Y, int imgs, int H, int W, int K, int stride, int N, int relu, hipStream_t s) {
  const int Ho = (H + 2 - 3) / stride + 1, Wo = (W + 2 - 3) / stride + 1;
  // 2-D-tile kernels for the MobileNet blocks they are instantiated for (K, N, stride)
  auto tile = [&](auto kern, int th, int tw) {
    hipLaunchKernelGGL(kern, dim3((Wo + tw - 1) / tw, (Ho + th - 1) / th, imgs), dim3(256), 0, s, (const bf16*)x,
                       (const uint32_t*)dw_w, dw_b, dw_relu, (const bf16*)Wt, bias, relu, (bf16*)Y, H, W, Ho, Wo);
  };
  // persistent form (dwpw_persist_kernel): grid = min(tiles, blocks-per-CU x CUs); VCX_DWPW_PERSIST=0
  // selects the one-tile-per-workgroup form
  static const bool persist = [] {
    const char* e = std::getenv("VCX_DWPW_PERSIST");
    return !(e && e[0] == '0');
  }();
  auto ptile = [&](auto kern, int th, int tw, int per_cu) {
    const int64_t tiles = (int64_t)((Wo + tw - 1) / tw) * ((Ho + th - 1) / th) * imgs;
    const int grid = (int)std::min<int64_t>(tiles, (int64_t)per_cu * vision_cus());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, s, (const bf16*)x, (const uint32_t*)dw_w, dw_b, dw_relu,
                       (const bf16*)Wt, bias, relu, (bf16*)Y, H, W, Ho, Wo, imgs);
  };
  if (persist && (int64_t)H * W * K * 2 < INT32_MAX && (int64_t)imgs * H * W < INT32_MAX) {
    if (K == 32 && N == 64 && stride == 1) return ptile(dwpw_persist_kernel<32, 64, 1, 8, 16>, 8, 16, 3);
    if (K == 64 && N == 128 && stride == 2) return ptile(dwpw_persist_kernel<64, 128, 2, 4, 16>, 4, 16, 2);
    if (K == 128 && N == 128 && stride == 1) return ptile(dwpw_persist_kernel<128, 128, 1, 4, 16>, 4, 16, 2);
  }
  if ((int64_t)H * W * K * 2 < INT32_MAX && imgs <= 65535 && (Ho + 3) / 4 <= 65535) {
    if (K == 32 && N == 64 && stride == 1) return tile(dwpw_tile_kernel<32, 64, 1, 8, 16>, 8, 16);
    if (K == 64 && N == 128 && stride == 2) return tile(dwpw_tile_kernel<64, 128, 2, 4, 16>, 4, 16);
    if (K == 128 && N == 128 && stride == 1) return tile(dwpw_tile_kernel<128, 128, 1, 4, 16>, 4, 16);
  }
  const int M = imgs * Ho * Wo;
  OutMap om{nullptr, N, 0, M, 0, 0, nullptr, 0, nullptr};
  ConvGeom cg{H, W, K, K, Ho, Wo, 3, stride, 1, 9 * K, (const uint32_t*)dw_w, dw_b, dw_relu};
  launch_gba<AM_DW>((const bf16*)x, (const bf16*)Wt, bias, (bf16*)Y, M, N, K, N, relu, om, cg, nullptr, 1, nullptr, s);
}

// conv1 (dw s1 + pw K1 -> N1) and conv2 (dw s2 + pw N1 -> N2) of MobileNet as ONE kernel
// (dwpw2_persist_kernel): x NHWC [imgs, H, W, K1] -> Y [imgs, Ho, Wo, N2], Ho = (H - 1) / 2 + 1.
// Returns false (nothing launched) for shapes without an instance.
bool vcx_dw_pw2(const void* x, const void* dw1_w, const float* dw1_b, int dw1_relu, const void* W1, const float* b1,
                int relu1, const void* dw2_w, const float* dw2_b, int dw2_relu, const void* W2, const float* b2,
                int relu2, void* Y, int imgs, int H, int W, int K1, int N1, int N2, hipStream_t s) {
  if (!(K1 == 32 && N1 == 64 && N2 == 128) || (int64_t)H * W * K1 * 2 >= INT32_MAX) return false;
  // tile geometry: VCX_DWPW2_TILE=8x8 (2 workgroups per CU, 79 KB LDS) or 4x8 (3 per CU, 52 KB: more
  // halo and conv1 recompute per output pixel, more workgroups to overlap the phases)
  static const int geo = [] {
    const char* e = std::getenv("VCX_DWPW2_TILE");
    return (e && std::string(e) == "4x8") ? 1 : 0;
  }();
  const int Ho = (H - 1) / 2 + 1, Wo = (W - 1) / 2 + 1;
  auto go = [&](auto kern, int lds, int th, int tw, int per_cu) {
    static bool attr_done = false;  // one attribute call per instance (the lambda is instantiated per kernel)
    if (!attr_done) {
      (void)hipFuncSetAttribute((const void*)kern, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
      attr_done = true;
    }
    const int64_t tiles = (int64_t)((Wo + tw - 1) / tw) * ((Ho + th - 1) / th) * imgs;
    const int grid = (int)std::min<int64_t>(tiles, (int64_t)per_cu * vision_cus());
    hipLaunchKernelGGL(kern, dim3(grid), dim3(256), lds, s, (const bf16*)x, (const uint32_t*)dw1_w, dw1_b, dw1_relu,
                       (const bf16*)W1, b1, relu1, (const uint32_t*)dw2_w, dw2_b, dw2_relu, (const bf16*)W2, b2, relu2,
                       (bf16*)Y, H, W, Ho, Wo, imgs);
  };
  if (geo == 1)
    go(dwpw2_persist_kernel<32, 64, 128, 4, 8, 3>, Dwpw2<32, 64, 128, 4, 8>::LDS, 4, 8, 3);
  else
    go(dwpw2_persist_kernel<32, 64, 128, 8, 8, 2>, Dwpw2<32, 64, 128, 8, 8>::LDS, 8, 8, 2);
  return true;
}

void vcx_gemm_bias_act(const void* X, const void* Wt, const float* bias, void* Y, int M, int N, int K, int ldy,
                       int relu, float* ws, int S, int* cnt, hipStream_t s) {
  vcx_gemm_bias_act_mapped(X, Wt, bias, Y, M, N, K, ldy, relu, nullptr, N, 0, M, 0, 0, ws, S, cnt, s);
}

void vcx_ssd_detect(const void* conf, const void* loc, const float* pri, const float* var, float* prob,
                    float* cls_out, int* cls_cnt, float* out, int* out_cnt, int N, int P, int C, int bg, float thresh,
                    float nms_thresh, int topk, int keep, hipStream_t s) {
  hipLaunchKernelGGL(ssd_softmax_kernel, dim3(stream_grid((int64_t)N * P, 256)), dim3(256), 0, s, (const bf16*)conf,
                     prob, N, P, C);
  hipLaunchKernelGGL(ssd_class_nms_kernel, dim3(N * (C - 1)), dim3(256), 0, s, prob, (const bf16*)loc, pri, var,
                     cls_out, cls_cnt, P, C, bg, thresh, nms_thresh, topk);
  hipLaunchKernelGGL(ssd_merge_kernel, dim3(N), dim3(256), 0, s, cls_out, cls_cnt, out, out_cnt, C, bg, topk, keep);
}

// Y4M 4:4:4 records of k annotated BGR frames [k, h, w, 3] on the GPU: per frame "FRAME\n" + the Y, U and
// V planes, laid out exactly as the file bytes (the requester's sink then only writes them). BT.601 full
// range with the host formulas' float operations in the same order and IEEE rounding at each step (plain
// operators under `fp contract(off)`: an fma would round once and move some bytes by one), so the bytes
// equal csrc/runtime/colour.cpp and io/video.py.
// One thread per pixel; the host conversion of a 100-frame chunk held the sink 16-25 ms per chunk
// (profiles/r5_video_job.txt).
__device__ __forceinline__ uint8_t sat_u8(float x) {
#pragma clang fp contract(off)
  x = x + 0.5f;
  x = x < 0.f ? 0.f : (x > 255.f ? 255.f : x);
  return (uint8_t)x;
}
__global__ void __launch_bounds__(256) bgr_to_y4m_kernel(const uint8_t* __restrict__ bgr, uint8_t* __restrict__ out,
                                                         int64_t n, int64_t total) {
#pragma clang fp contract(off)
  const int64_t rec = 6 + 3 * n;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t f = i / n, px = i - f * n;
    const uint8_t* src = bgr + 3 * i;
    const float b = src[0], g = src[1], r = src[2];
    const float y = 0.299f * r + 0.587f * g + 0.114f * b;
    uint8_t* o = out + f * rec + 6;
    o[px] = sat_u8(y);
    o[n + px] = sat_u8((b - y) * 0.564f + 128.0f);
    o[2 * n + px] = sat_u8((r - y) * 0.713f + 128.0f);
    if (px < 6) out[f * rec + px] = (uint8_t)("FRAME\n"[px]);
  }
}

void vcx_bgr_to_y4m(const uint8_t* bgr, uint8_t* out, int k, int w, int h, hipStream_t s) {
  const int64_t n = (int64_t)w * h, total = n * k;
  hipLaunchKernelGGL(bgr_to_y4m_kernel, dim3(stream_grid(total, 256)), dim3(256), 0, s, bgr, out, n, total);
}

void vcx_annotate(uint8_t* frames, int N, int h, int w, const float* dets, const int* det_cnt, int keep, int label,
                  float thresh, uint32_t box_bgr, const uint8_t* name_mask, int nm_h, int nm_w, int nm_x, int nm_y,
                  uint32_t name_bgr, const uint8_t* lab_masks, int lm_n, int lm_h, int lm_w, int lm_x, int lm_y,
                  uint32_t lab_bgr, int* counts_out, hipStream_t s) {
  hipLaunchKernelGGL(annotate_kernel, dim3(N), dim3(256), 0, s, frames, h, w, dets, det_cnt, keep, label, thresh,
                     box_bgr, name_mask, nm_h, nm_w, nm_x, nm_y, name_bgr, lab_masks, lm_n, lm_h, lm_w, lm_x, lm_y,
                     lab_bgr, counts_out);
}
