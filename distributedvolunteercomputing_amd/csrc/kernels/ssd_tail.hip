// MobileNet-SSD tail in ONE launch: the SSD extras (conv14_1 .. conv17_2) and all six multibox heads
// (prototxt 891-1775; SURVEY.md K7 + K8).
//
// Why (profiles/r3_detector_chunk_final.txt): per 100-frame chunk the tail was ~20 launches of small
// split-K GEMMs and reductions (M = 100 x 25 .. 100 x 1 rows) plus the side-stream head GEMMs:
// about 330 us of the 1.30 ms chunk for ~4 % of its FLOPs, latency-bound on launch boundaries and
// k-loops, with ~85 us of host-bound idle GPU before DetectionOutput.
//
// Here every frame's extras chain is independent of every other frame's, so one launch holds:
//   * role A, one workgroup per frame: conv14_1 -> conv14_2 (+ its heads) -> conv15_1 -> ... ->
//     conv17_2 (+ its heads), layer after layer with only a workgroup barrier in between (each
//     layer's output is written to its NHWC tensor and read back by the same workgroup from L2);
//   * role B, the two wide heads (sources conv11 19x19 and conv13 10x10, all frames as one GEMM
//     each), split into 64 x 128 output tiles over the remaining workgroups.
// One tile routine serves all: out[64 x 128] of act(A W^T + b), A either the rows of an NHWC tensor
// (1x1 convolution) or gathered on the fly (3x3 stride 2 pad 1 implicit GEMM, 16-B taps); 8 waves
// as 2 x 4, 32 x 32 per wave on v_mfma_f32_16x16x32_bf16 (two waves per SIMD hide each other's waits); K in steps of 128 (four 32-deep LDS
// slices, XOR-swizzled 64-B rows), register-staged two steps ahead through three register sets
// (these k-loops are short and L2/MALL-latency-bound: with 64-deep steps and one step of lookahead
// the tail took 433 us per 100-frame chunk, profiles/r4_detector_chunk.txt). Head outputs are written
// straight into the concatenated mbox_loc / mbox_conf buffers (Permute + Flatten + Concat as
// address arithmetic, as the per-layer head GEMM does).
#include "vcx_common.h"

namespace vcx {
namespace ssd_tail {

typedef short sx8 __attribute__((ext_vector_type(8)));

constexpr int TBM = 64, TBN = 128, SLK = 32, STEPK = 128, NTH = 512;
constexpr int MAXL = 16;

// kind: 0 = 1x1 convolution (+bias, act) -> NHWC Y;  1 = 3x3 stride-2 pad-1 convolution -> NHWC Y;
//       2 = 1x1 multibox head: columns < split -> Y (loc), >= split -> Y2 (conf), per image rows
//           of `split` / `N - split` values at image strides ys1 / ys2
struct Layer {
  const bf16* X;    // input NHWC [imgs, H, W, C]
  const bf16* Wt;   // [N, K] (K = C for 1x1; 9 C, (ky, kx, c) order, for 3x3)
  const float* b;   // [N]
  bf16* Y;
  bf16* Y2;
  int H, W, C, Ho, Wo, N, K, kind, relu, split;
  long long ys1, ys2;
};
struct Plan {
  Layer L[MAXL];
  int nchain;      // layers 0 .. nchain-1: the per-frame chain (role A)
  int nlayers;     // layers nchain .. nlayers-1: wide heads over all frames (role B)
  int frames;      // role A workgroups
  int tiles_start[MAXL + 1];  // role B: prefix sums of the wide layers' tile counts
};

__device__ __forceinline__ int gswz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }
__device__ __forceinline__ int sidx(int row, int chunk) { return row * SLK + ((chunk ^ gswz(row)) << 3); }

// LDS: 2 buffers x (A 64 x 128 + B 128 x 128) bf16 = 96 KB
constexpr int A_ELEMS = TBM * STEPK, B_ELEMS = TBN * STEPK, BUF_ELEMS = A_ELEMS + B_ELEMS;

// one 64 x 128 output tile of layer Lr for the image range starting at img0: rows m0 .. m0+63 of the
// M rows (M = Ho * Wo for one frame in role A; imgs * Ho * Wo in role B), columns n0 .. n0+127
__device__ void run_tile(bf16* smem, const Layer& Lr, int img0, int M, int m0, int n0) {
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 2, wn = wid & 3;  // 8 waves as 2 (M) x 4 (N): 32 x 32 per wave
  const int K = Lr.K, N = Lr.N, C = Lr.C;
  const bool conv3 = Lr.kind == 1;
  const int pix = Lr.Ho * Lr.Wo;
  // staging: each step moves A 64 x 128 (1024 16-B chunks: 2 per thread) and B 128 x 128 (4 per
  // thread); chunk e = tid + 512 i: row e >> 4, k offset (e & 15) * 8 (slice (e & 15) >> 2). Columns
  // past K (a K that is not a multiple of 128, e.g. conv17_2's 576) load as zero.
  const int kc = (tid & 15) * 8;
  int arow_ok[2], arow_iy[2], arow_ix[2];
  const bf16* arow_ptr[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int gm = m0 + (tid >> 4) + 32 * i;
    arow_ok[i] = gm < M ? 1 : 0;
    const int g2 = gm < M ? gm : 0;
    const int im = g2 / pix, p = g2 - im * pix, oy = p / Lr.Wo, ox = p - oy * Lr.Wo;
    arow_iy[i] = oy * 2 - 1;
    arow_ix[i] = ox * 2 - 1;
    // 1x1: the input row (same pixel grid); 3x3: the image base
    arow_ptr[i] = conv3 ? Lr.X + (size_t)(img0 + im) * Lr.H * Lr.W * C : Lr.X + ((size_t)img0 * pix + g2) * C;
  }
  const int cshift = 31 - __builtin_clz(C);  // C is a power of two (host check)
  auto loadA = [&](int i, int k) -> sx8 {
    if (!arow_ok[i] || k >= K) return sx8{0, 0, 0, 0, 0, 0, 0, 0};
    if (!conv3) return *(const sx8*)(arow_ptr[i] + k);
    const int tap = k >> cshift, c = k & (C - 1), ky = tap / 3, kx = tap - ky * 3;
    const int iy = arow_iy[i] + ky, ix = arow_ix[i] + kx;
    if (iy < 0 || iy >= Lr.H || ix < 0 || ix >= Lr.W) return sx8{0, 0, 0, 0, 0, 0, 0, 0};
    return *(const sx8*)(arow_ptr[i] + (iy * Lr.W + ix) * C + c);
  };
  auto loadB = [&](int i, int k) -> sx8 {
    const int gn = n0 + (tid >> 4) + 32 * i;
    return gn < N && k < K ? *(const sx8*)(Lr.Wt + (size_t)gn * K + k) : sx8{0, 0, 0, 0, 0, 0, 0, 0};
  };
  struct Regs {
    sx8 a[2], b[4];
  };
  auto gload = [&](Regs& r, int step) {
    const int k = step * STEPK + kc;
#pragma unroll
    for (int i = 0; i < 2; ++i) r.a[i] = loadA(i, k);
#pragma unroll
    for (int i = 0; i < 4; ++i) r.b[i] = loadB(i, k);
  };
  const int sl = kc >> 5, ch = (kc & 31) >> 3;
  auto sstore = [&](const Regs& r, int buf) {
    bf16* sA = smem + buf * BUF_ELEMS + sl * TBM * SLK;
    bf16* sB = smem + buf * BUF_ELEMS + A_ELEMS + sl * TBN * SLK;
#pragma unroll
    for (int i = 0; i < 2; ++i) *(sx8*)(sA + sidx((tid >> 4) + 32 * i, ch)) = r.a[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) *(sx8*)(sB + sidx((tid >> 4) + 32 * i, ch)) = r.b[i];
  };
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const int fr = lane & 15, fc = lane >> 4;
  auto compute = [&](int buf) {
#pragma unroll
    for (int s = 0; s < STEPK / SLK; ++s) {
      const bf16* sA = smem + buf * BUF_ELEMS + s * TBM * SLK;
      const bf16* sB = smem + buf * BUF_ELEMS + A_ELEMS + s * TBN * SLK;
      sx8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) af[i] = *(const sx8*)(sA + sidx(wm * 32 + i * 16 + fr, fc));
#pragma unroll
      for (int j = 0; j < 2; ++j) bfr[j] = *(const sx8*)(sB + sidx(wn * 32 + j * 16 + fr, fc));
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[j], af[i], acc[i][j], 0, 0, 0);
    }
  };
  // three register sets, loads issued two steps ahead of their LDS store (these k-loops are short
  // and L2/MALL-latency-bound); two LDS buffers. Step k: load step k + 2 into set (k + 2) % 3 (its
  // step k - 1 data went to LDS during step k - 2), compute buffer k % 2, store set (k + 1) % 3 into
  // buffer (k + 1) % 2 (last read by step k - 1, before the previous barrier), barrier.
  const int nk = (K + STEPK - 1) / STEPK;
  Regs r0, r1, r2;
  gload(r0, 0);
  if (nk > 1) gload(r1, 1);
  sstore(r0, 0);
  __syncthreads();
#define VCX_TAIL_STEP(KK, RL, RS, BC, BS)            \
  {                                                  \
    const int k_ = (KK);                             \
    if (k_ >= nk) break;                             \
    if (k_ + 2 < nk) gload(RL, k_ + 2);              \
    compute(BC);                                     \
    if (k_ + 1 < nk) sstore(RS, BS);                 \
    __syncthreads();                                 \
  }
  for (int k = 0; k < nk; k += 6) {
    VCX_TAIL_STEP(k + 0, r2, r1, 0, 1)
    VCX_TAIL_STEP(k + 1, r0, r2, 1, 0)
    VCX_TAIL_STEP(k + 2, r1, r0, 0, 1)
    VCX_TAIL_STEP(k + 3, r2, r1, 1, 0)
    VCX_TAIL_STEP(k + 4, r0, r2, 0, 1)
    VCX_TAIL_STEP(k + 5, r1, r0, 1, 0)
  }
#undef VCX_TAIL_STEP
  // epilogue: lane holds 4 consecutive columns of one row per (i, j)
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int gn = n0 + wn * 32 + j * 16 + 4 * (lane >> 4);
    float bv[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) bv[r] = gn + r < N ? Lr.b[gn + r] : 0.f;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int gm = m0 + wm * 32 + i * 16 + (lane & 15);
      if (gm >= M) continue;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        v[r] = acc[i][j][r] + bv[r];
        if (Lr.relu) v[r] = fmaxf(v[r], 0.f);
      }
      if (Lr.kind != 2) {
        bf16* q = Lr.Y + ((size_t)img0 * pix + gm) * N + gn;
        if (gn + 3 < N) {
          *(bf16x4*)q = bf16x4{(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
        } else {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (gn + r < N) q[r] = (bf16)v[r];
        }
      } else {
        const int im = gm / pix, p = gm - im * pix;
        const int nl = Lr.split, nc = N - Lr.split;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int n = gn + r;
          if (n >= N) break;
          if (n < nl)
            Lr.Y[(size_t)(img0 + im) * Lr.ys1 + p * nl + n] = (bf16)v[r];
          else
            Lr.Y2[(size_t)(img0 + im) * Lr.ys2 + p * nc + (n - nl)] = (bf16)v[r];
        }
      }
    }
  }
  __syncthreads();  // the next tile restages the same LDS buffers
}

__global__ void __launch_bounds__(NTH) ssd_tail_kernel(Plan P) {
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * BUF_ELEMS];
  const int bid = blockIdx.x;
  if (bid < P.frames) {  // role A: frame `bid` through the whole chain
    for (int l = 0; l < P.nchain; ++l) {
      const Layer& Lr = P.L[l];
      const int M = Lr.Ho * Lr.Wo;
      for (int m0 = 0; m0 < M; m0 += TBM)
        for (int n0 = 0; n0 < Lr.N; n0 += TBN) run_tile(smem, Lr, bid, M, m0, n0);
      // this layer's outputs (global stores of every wave) before the next layer reads them
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __syncthreads();
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
    }
    return;
  }
  // role B: one tile of a wide head (all frames as one GEMM)
  int t = bid - P.frames;
  for (int l = P.nchain; l < P.nlayers; ++l) {
    const int lo = P.tiles_start[l - P.nchain], hi = P.tiles_start[l - P.nchain + 1];
    if (t < hi) {
      const Layer& Lr = P.L[l];
      const int ntn = (Lr.N + TBN - 1) / TBN;
      const int tt = t - lo;
      run_tile(smem, Lr, 0, P.frames * Lr.Ho * Lr.Wo, (tt / ntn) * TBM, (tt % ntn) * TBN);
      return;
    }
  }
}

}  // namespace ssd_tail
}  // namespace vcx

using namespace vcx;

// layer records: 13 ints per layer (kind, H, W, C, Ho, Wo, N, K, relu, split, ys1, ys2, unused) and
// 5 pointers (X, Wt, b, Y, Y2); returns false if the plan does not fit the kernel
bool vcx_ssd_tail(int nchain, int nlayers, int frames, const long long* ints, const void* const* ptrs, hipStream_t s) {
  using namespace ssd_tail;
  if (nlayers > MAXL || nchain > nlayers || frames <= 0) return false;
  Plan P{};
  P.nchain = nchain;
  P.nlayers = nlayers;
  P.frames = frames;
  int tiles = 0;
  P.tiles_start[0] = 0;
  for (int l = 0; l < nlayers; ++l) {
    const long long* q = ints + 13 * l;
    Layer& L = P.L[l];
    L.kind = (int)q[0];
    L.H = (int)q[1];
    L.W = (int)q[2];
    L.C = (int)q[3];
    L.Ho = (int)q[4];
    L.Wo = (int)q[5];
    L.N = (int)q[6];
    L.K = (int)q[7];
    L.relu = (int)q[8];
    L.split = (int)q[9];
    L.ys1 = q[10];
    L.ys2 = q[11];
    L.X = (const bf16*)ptrs[5 * l + 0];
    L.Wt = (const bf16*)ptrs[5 * l + 1];
    L.b = (const float*)ptrs[5 * l + 2];
    L.Y = (bf16*)ptrs[5 * l + 3];
    L.Y2 = (bf16*)ptrs[5 * l + 4];
    if (L.K % 32 || L.C % 8 || (L.C & (L.C - 1)) || (L.kind == 1 ? L.K != 9 * L.C : L.K != L.C)) return false;
    if (L.kind == 2 && (L.split <= 0 || L.split >= L.N)) return false;
    if (l >= nchain) {
      tiles += ((frames * L.Ho * L.Wo + TBM - 1) / TBM) * ((L.N + TBN - 1) / TBN);
      P.tiles_start[l - nchain + 1] = tiles;
    }
  }
  hipLaunchKernelGGL(ssd_tail_kernel, dim3(frames + tiles), dim3(NTH), 0, s, P);
  return true;
}
