// Forward / input-gradient GEMM for gfx950 on gemm_wg's staging pipeline:
//
//   C[M, N] = A[M, K] . B[N, K]^T (+ bias[N])     (both operands K-contiguous: x W^T, dY (W^T)^T)
//
// the plain forward GEMMs and the LM head's input gradient are the last library GEMMs of the
// GPT-2 step. Structure:
//   * 256 x 256 tile per workgroup in one of two wave layouts: 8 waves as 2 (M) x 4 (N) of 128 x 64 (two waves per
//     SIMD, 128 accumulators in VGPRs; the default) or 4 waves as 2 x 2 of 128 x 128 (hipBLASLt's MT256x256x64
//     WG32_8_1 / MIWT8_8 geometry: one wave per SIMD, 256 accumulators in AGPRs); for N = 128 / 64 a 256 x 128
//     tile (8 waves of 64 x 64) / 256 x 64 tile (4 waves of 64 x 64, two workgroups per CU);
//   * CONV: a 3x3 convolution (pad 1, stride 1 | 2) as an implicit GEMM -- the patch matrix of NHWC x gathered by
//     the LDS-DMA's per-lane source offsets, padding taps as offsets past the buffer resource (the load returns 0);
//     the ResNet-50 3x3 forwards and stride-1 input gradients (models/resnet.py, 1.09-1.38x MIOpen at every
//     stage, profiles/r6_conv3x3_fwd.txt);
//   * split-K over one round of workgroups for deep-K / few-tile shapes: fp32 partials straight from the
//     accumulators, summed with the bias by splitk_bias_kernel;
//   * 4-slot LDS ring of 32-deep K-slices (32 KB each: A 256 x 64 B, B 256 x 64 B), LDS-DMA issued as inline asm
//     (hipcc's waitcnt pass cannot see it, so it adds no vmcnt drains), a counted vmcnt that keeps two slices in
//     flight across every raw s_barrier, fragments of slice s + 1 read during slice s into a second register set;
//   * MFMAs as inline asm on pinned accumulators (the builtin let the register allocator rotate them: 68
//     v_accvgpr_mov per 128 MFMAs in the 4-wave loop);
//   * 16-B chunks XOR-swizzled per row F[(row >> 2) & 3] = {0, 2, 3, 1} (gemm.hip), applied to the DMA's per-lane
//     SOURCE address since the DMA writes each wave's 1-KB piece lane-linearly: conflict-free ds_read_b128;
//   * optional bias added in the epilogue (F.linear's GemmAndBias);
//   * the output tile leaves through the (then idle) ring as whole row segments, non-temporal stores;
//   * XCD-aware tile order: each XCD's concurrent tiles form a block of GROUP_M row panels x column panels.
// Measured (profiles/r6_gemm_f.txt, GPT-2 shapes at 65536 tokens): 0.85-0.93x the library (8 waves: qkv 227.9 vs
// 203.6 us, fc2 259.0 vs 218.6, 4096^3 1317 vs 1518 TF/s -- the cdna guide's 8-phase template level); 4 waves
// 0.78-0.81x. Counters (8 waves, qkv + 4096^3): MFMA busy 48 %, 36 % of wave-cycles parked at waits / barriers,
// against the library's 57 % / 14 %; a 5-slot ring (memory latency) and staggering the two M halves' DMA issue
// measured even. Hence opt-in for the linear layers (config.gemm_fwd = "vcx"); the library keeps the GPT-2 forward
// GEMMs, while the convolutions -- where MIOpen's kernels run at 300-600 TF/s -- default to this kernel.
// Reference analog: per-frame net.forward, /root/reference/worker.py:248-249 (the pointwise GEMMs).
#include <type_traits>

#include "vcx_common.h"

namespace vcx {
namespace gemm_f {

typedef short sx8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BKS = 32;
constexpr int ROWB = BKS * 2;           // 64 B per row per slice
constexpr int SLOT_A = BM * ROWB;       // 16 KB: the A slice

__device__ __forceinline__ int swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

// buffer resource words over [base, base + bytes): wave-uniform base and size (SGPRs), 32-bit per-lane offsets
__device__ __forceinline__ u32x4 desc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  return u32x4{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}

// one 1-KB LDS-DMA piece (16 B per lane to LDS base + 16 lane), M0 = the LDS byte address; `s_nop 0`: the
// M0 write -> LDS-DMA hazard
__device__ __forceinline__ void dma16(u32x4 d, int voff, int soff, const char* lds) {
  const unsigned m0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) char*)lds;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(d), "s"(soff), "{m0}"(m0)
               : "memory");
}

// s_waitcnt vmcnt(N) lgkmcnt(0) for N up to 63 (vmcnt bits [3:0] and [15:14])
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  __builtin_amdgcn_s_waitcnt(0x0070 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

// Tile 256 x BNT, WM waves along M and WN along N: <2, 2, 256> = 4 waves of 128 x 128 (one wave per SIMD, 256
// accumulator registers), <2, 4, 256> = 8 waves of 128 x 64 (two waves per SIMD, 128; the default),
// <4, 2, 128> = 8 waves of 64 x 64 for 128 output columns (the 128-channel convolutions)
template <int WM_, int WN_, int BNT_>
struct Geo {
  static constexpr int WM = WM_, WN = WN_, BNT = BNT_, WAVES = WM * WN, NT = 64 * WAVES;
  static constexpr int TM = BM / WM, IB = TM / 16;  // output rows per wave, A fragments (row blocks) per wave
  static constexpr int TN = BNT / WN, JB = TN / 16;  // output columns per wave, B fragments per wave
  static constexpr int AOPS = 16 / WAVES, BOPS = BNT / 16 / WAVES;  // LDS-DMA pieces per wave per slice
  static constexpr int OPS = AOPS + BOPS, OPG = (OPS + 3) / 4;      // ... and per MFMA group (first 4 groups)
  static constexpr int SLOT = SLOT_A + BNT * ROWB;  // A and B slices
  static constexpr int RB = TN * 2;                 // staged output row bytes
  static constexpr int CPR = RB / 16;               // 16-B chunks per staged row
  static_assert(AOPS * WAVES == 16 && BOPS * WAVES == BNT / 16 && JB <= IB && IB <= 8, "tile geometry");
};
using G4 = Geo<2, 2, 256>;
using G8 = Geo<2, 4, 256>;
using G8n = Geo<4, 2, 128>;
using G4n = Geo<4, 1, 64>;  // 4 waves of 64 x 64 on a 256 x 64 tile (64 output channels; 2 workgroups per CU)

template <class G>
struct Frags {
  sx8 a[G::IB];  // A fragments: the wave's row blocks of 16 (output rows)
  sx8 b[G::JB];  // B fragments: the wave's column blocks of 16
};

// 3x3 convolution (pad 1) as an implicit GEMM: A = the patch matrix of NHWC x gathered while staging
struct Conv {
  int H, W, lc, Ho, Wo, stride;  // lc = log2(Cin)
  int flip;                       // gather tap (2 - ky, 2 - kx) for weight tap (ky, kx): w[Cin][ky][kx][Cout] unflipped
  int btap;                       // > 0: B is tap-major, [9][N][Cin] (ldb = Cin), tap t's rows at t * btap elements
  unsigned xbytes;
};

// D: ring slots, two slices in flight across each barrier (a 5-slot ring over the whole 160 KB LDS, three in
// flight, measured even to 4 % slower: 236.3 vs 227.9 us qkv, 105.7 vs 104.4 sq4096)
// CONV: A is NHWC x [imgs, H, W, Cin] and row m of the GEMM the output pixel m of [imgs, Ho, Wo]; K = 9 Cin in the
// [ky][kx][Cin] order of the channels-last weight, each 32-deep slice inside one tap (Cin a power of two >= 64)
template <class G, int D, bool CONV>
__global__ void __launch_bounds__(G::NT, 1)
    gemm_f_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
                  const bf16* __restrict__ bias, int M, int N, int K, int lda, int ldb, int ldc, int tilesN,
                  Conv cv, int splits, float* __restrict__ ws) {
  static_assert(D == 4, "the pipeline tail below is written for a 4-slot ring");
  constexpr int IB = G::IB, JB = G::JB, OPS = G::OPS, AOPS = G::AOPS, WAVES = G::WAVES, WN = G::WN, TM = G::TM;
  constexpr int BN = G::BNT, SLOT = G::SLOT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / WN, wn = wid % WN;

  // ---- XCD-aware bijective tile order (gemm.hip): consecutive logical tiles share an XCD, walked as blocks of
  // GROUP_M row panels x all column panels
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wga = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  // split-K: the grid is splits x tiles, split-major (one XCD's neighbours share the split's K range)
  const int tiles = nwg / splits, split = wga / tiles, wg = wga - split * tiles;
  const int ks0 = split * (K / BKS / splits);  // the split's first K slice
  constexpr int GROUP_M = 4;
  const int tilesM = tiles / tilesN;
  const int per_group = GROUP_M * tilesN;
  const int gfirst = (wg / per_group) * GROUP_M;
  const int gsize = min(tilesM - gfirst, GROUP_M);
  const int m0 = (gfirst + (wg % per_group) % gsize) * BM, n0 = ((wg % per_group) / gsize) * BN;

  // ---- staging: piece p (0..15) of an operand slice = rows 16 p .. 16 p + 15 (64 lanes x 16 B); wave w moves
  // pieces w + WAVES q (q < HOPS) of A and of B. Lane l: row 16 p + (l >> 2), physical chunk l & 3 holding
  // logical chunk (l & 3) ^ F(row) (F depends on row bits 2..3 only: the same for every piece). Rows past the
  // operand (ragged M, the half column panel of N % 256 == 128) read past the resource: zeros, and their
  // outputs are never stored.
  const int prow = lane >> 2, pch = (lane & 3) ^ swz(prow);
  const int rowsA = min(BM, M - m0), rowsB = min(BN, N - n0);
  const u32x4 ra = CONV ? desc(A, cv.xbytes) : desc(A + (int64_t)m0 * lda, (unsigned)(((int64_t)(rowsA - 1) * lda + K) * 2));
  const u32x4 rb = desc(B + (int64_t)n0 * ldb, (unsigned)(((CONV && cv.btap ? 8 * (int64_t)cv.btap + (1 << cv.lc)
                                                                            : (int64_t)K) +
                                                             (int64_t)(rowsB - 1) * ldb) * 2));
  int va[AOPS], vb[G::BOPS];
  // CONV: per A piece the lane's output pixel as the input pixel of tap (0, 0) -- (ih0, iw0) and its index pix0
  // (rows past M: ih0 = -4, never inside the image)
  int ih0[AOPS], iw0[AOPS];
#pragma unroll
  for (int q = 0; q < AOPS; ++q) {
    const int r = (wid + WAVES * q) * 16 + prow;
    if constexpr (CONV) {
      const int m = m0 + r, hw = cv.Ho * cv.Wo;
      const int n = m / hw, oh = (m - n * hw) / cv.Wo, ow = m - n * hw - oh * cv.Wo;
      ih0[q] = m < M ? oh * cv.stride - 1 : -4;
      iw0[q] = ow * cv.stride - 1;
      va[q] = (n * cv.H + ih0[q]) * cv.W + iw0[q];
    } else {
      va[q] = r < rowsA ? (r * lda + pch * 8) * 2 : 0x7fffff00;  // past the resource: returns 0
    }
  }
#pragma unroll
  for (int q = 0; q < G::BOPS; ++q) {
    const int r = (wid + WAVES * q) * 16 + prow;
    vb[q] = r < rowsB ? (r * ldb + pch * 8) * 2 : 0x7fffff00;
  }
  auto stage_op = [&](int s, int o) {  // op o of slice s: A piece q = o (o < AOPS), B piece q = o - AOPS
    char* slot = smem + (s % D) * SLOT;
    const int q = o < AOPS ? o : o - AOPS;
    if (o < AOPS) {
      if constexpr (CONV) {  // slice s = channels c0 .. c0 + 31 of tap t = (ky, kx); padding taps read zeros
        const int sg = ks0 + s;  // the global slice
        const int t = (sg * BKS) >> cv.lc, c0 = (sg * BKS) & ((1 << cv.lc) - 1);
        int ky = (t * 11) >> 5, kx = t - 3 * ky;  // t / 3 for t < 9
        if (cv.flip) ky = 2 - ky, kx = 2 - kx;     // an input gradient against the unflipped transposed weight
        const int ih = ih0[q] + ky, iw = iw0[q] + kx;
        const bool ok = (unsigned)ih < (unsigned)cv.H && (unsigned)iw < (unsigned)cv.W;
        const int voff = ok ? (((va[q] + ky * cv.W + kx) << cv.lc) + c0 + pch * 8) * 2 : 0x7fffff00;
        dma16(ra, voff, 0, slot + (wid + WAVES * q) * 1024);
      } else {
        dma16(ra, va[q], (ks0 + s) * ROWB, slot + (wid + WAVES * q) * 1024);
      }
    } else {
      int soff = (ks0 + s) * ROWB;
      if constexpr (CONV) {
        if (cv.btap) {  // tap-major B (the transposed weight of an input gradient): tap t's rows at t * btap
          const int sg = ks0 + s;
          const int t = (sg * BKS) >> cv.lc, c0 = (sg * BKS) & ((1 << cv.lc) - 1);
          soff = (t * cv.btap + c0) * 2;
        }
      }
      dma16(rb, vb[q], soff, slot + SLOT_A + (wid + WAVES * q) * 1024);
    }
  };
  auto stage = [&](int s) {
#pragma unroll
    for (int o = 0; o < OPS; ++o) stage_op(s, o);
  };

  // ---- fragment reads: lane l -> row (l & 15) of a 16-row block, k chunk (l >> 4)
  const int frow = lane & 15;
  const int foff = frow * ROWB + (((lane >> 4) ^ swz(frow)) << 4);
  auto afrag = [&](int s, int i) {
    return *(const sx8*)(smem + (s % D) * SLOT + (wm * TM + 16 * i) * ROWB + foff);
  };
  auto bfrag = [&](int s, int j) {
    return *(const sx8*)(smem + (s % D) * SLOT + SLOT_A + (wn * G::TN + 16 * j) * ROWB + foff);
  };

  f32x4 acc[IB][JB];
#pragma unroll
  for (int i = 0; i < IB; ++i)
#pragma unroll
    for (int j = 0; j < JB; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // in-place accumulation, the accumulators pinned by the constraint (with the builtin the register allocator
  // rotated them through 68 v_accvgpr_mov per 128 MFMAs): AGPRs at one wave per SIMD, VGPRs at two (the
  // unified file split 128 / 128 would not fit the fragments). An accumulate chain needs no wait states; the
  // epilogue's first reads are padded by hand (the MFMAs are invisible to hipcc's hazard recognizer).
  auto mma_row = [&](const Frags<G>& f, int i) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      if constexpr (G::WAVES == 4)
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc[i][j]) : "v"(f.b[j]), "v"(f.a[i]));
      else
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i][j]) : "v"(f.b[j]), "v"(f.a[i]));
    }
    __builtin_amdgcn_s_setprio(0);
  };

  // one step: slice s in fc; make slice s + 1 visible (the counted vmcnt leaves the D - 2 slices behind it in
  // flight), issue slice s + D into the slot of slice s (read into registers during step s - 1), then 8 MFMA
  // groups (one output row block each), each followed by the reads of slice s + 1's fragments of that row (and
  // column) block into fn; the DMA ops ride along the first 4 groups (placing the second M half's in the last 4
  // measured even, 8 waves: 233.5 vs 234.3 us qkv, 109.2 vs 110.1 sq4096)
  auto step = [&](int s, Frags<G>& fc, Frags<G>& fn, auto STAGE, auto PEND) {
    wait_vm<decltype(PEND)::value>();
    barrier();
#pragma unroll
    for (int g = 0; g < IB; ++g) {
      if constexpr (decltype(STAGE)::value) {
#pragma unroll
        for (int o = G::OPG * g; o < G::OPG * (g + 1); ++o)
          if (o < OPS) stage_op(s + D, o);
      }
      __builtin_amdgcn_sched_barrier(0);
      mma_row(fc, g);
      __builtin_amdgcn_sched_barrier(0);
      fn.a[g] = afrag(s + 1, g);
      if (g < JB) fn.b[g] = bfrag(s + 1, g);
    }
  };

  using T = std::true_type;
  using F = std::false_type;
  using PS = std::integral_constant<int, (D - 2) * OPS>;
  using P2 = std::integral_constant<int, 2 * OPS>;
  using P1 = std::integral_constant<int, OPS>;
  using P0 = std::integral_constant<int, 0>;
  const int nk = K / BKS / splits;  // slices per split: even, >= 6 (host)
  Frags<G> f0, f1;
#pragma unroll
  for (int t = 0; t < D; ++t) stage(t);
  wait_vm<(D - 1) * OPS>();  // slice 0 landed
  barrier();
#pragma unroll
  for (int g = 0; g < IB; ++g) f0.a[g] = afrag(0, g);
#pragma unroll
  for (int j = 0; j < JB; ++j) f0.b[j] = bfrag(0, j);
  int s = 0;
#pragma unroll 1
  for (; s + D + 1 < nk; s += 2) {  // both steps stage
    step(s, f0, f1, T{}, PS{});
    step(s + 1, f1, f0, T{}, PS{});
  }
  // s = nk - 4: three steps, nothing left to stage
  step(s, f0, f1, F{}, P2{});
  step(s + 1, f1, f0, F{}, P1{});
  step(s + 2, f0, f1, F{}, P0{});
#pragma unroll
  for (int g = 0; g < IB; ++g) mma_row(f1, g);

  // ---- epilogue: acc[i][j] = C[wm 128 + 16 i + (l & 15)][wn TN + 16 j + 4 (l >> 4) .. + 3]. Each wave stages
  // its 128 x TN bf16 block in its own part of the ring (RB-byte rows, 16-B chunks XOR-swizzled by the row),
  // then writes whole RB-byte row segments (CPR lanes per row) with non-temporal stores.
  // the last MFMAs' results -> their first readers: >= 12 wait states for an 8-pass MFMA
  asm volatile("s_nop 7\n\ts_nop 7" ::: "memory");
  __syncthreads();  // every wave is past its last fragment read; every DMA retired (vmcnt(0) of the last step)
  if (n0 + wn * G::TN >= N) return;  // the missing half of a 128-column last panel (no barrier follows)
  if (splits > 1) {  // fp32 partial straight from the accumulators (splitk_bias_kernel sums them)
    float* const wb = ws + ((int64_t)split * M + m0 + wm * TM) * N + n0 + wn * G::TN + 4 * (lane >> 4);
    const int mrem = M - (m0 + wm * TM);
#pragma unroll
    for (int i = 0; i < IB; ++i) {
      const int r = 16 * i + (lane & 15);
      if (r < mrem) {
#pragma unroll
        for (int j = 0; j < JB; ++j) *(f32x4*)(wb + (int64_t)r * N + 16 * j) = acc[i][j];
      }
    }
    return;
  }
  constexpr int RB = G::RB, CPR = G::CPR;
  char* const stg = smem + wid * (TM * RB);
  float bv[JB][4];  // the bias of the lane's output columns (zeros without one)
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    bf16x4 b4 = {};
    if (bias) b4 = *(const bf16x4*)(bias + n0 + wn * G::TN + 16 * j + 4 * (lane >> 4));
#pragma unroll
    for (int t = 0; t < 4; ++t) bv[j][t] = (float)b4[t];
  }
#pragma unroll
  for (int i = 0; i < IB; ++i) {
    const int r = 16 * i + (lane & 15);
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int c = 16 * j + 4 * (lane >> 4);
      bf16x4 v;
#pragma unroll
      for (int t = 0; t < 4; ++t) v[t] = (bf16)(acc[i][j][t] + bv[j][t]);
      *(bf16x4*)(stg + r * RB + (((c >> 3) ^ (r & (CPR - 1))) << 4) + ((c >> 2) & 1) * 8) = v;
    }
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the wave reads back only its own block
  const int k = lane % CPR;
  const int mrem = M - (m0 + wm * TM);
  bf16* const base = C + (int64_t)(m0 + wm * TM) * ldc + n0 + wn * G::TN + k * 8;
#pragma unroll 8
  for (int it = 0; it < TM / (64 / CPR); ++it) {
    const int r = it * (64 / CPR) + lane / CPR;
    const bf16x8 v = *(const bf16x8*)(stg + r * RB + ((k ^ (r & (CPR - 1))) << 4));
    if (r < mrem) __builtin_nontemporal_store(v, (bf16x8*)(base + (int64_t)r * ldc));
  }
}

// C[m][n] = bf16(sum over splits of ws[s][m][n] (+ bias[n])), 4 columns per thread
__global__ void __launch_bounds__(256) splitk_bias_kernel(const float* __restrict__ ws, const bf16* __restrict__ bias,
                                                        bf16* __restrict__ C, int M, int N, int ldc, int splits) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4, mn = (int64_t)M * N;
  if (i >= mn) return;
  const int m = (int)(i / N), n = (int)(i - (int64_t)m * N);
  f32x4 a = *(const f32x4*)(ws + i);
  for (int s = 1; s < splits; ++s) a += *(const f32x4*)(ws + (int64_t)s * mn + i);
  bf16x4 b4 = {};
  if (bias) b4 = *(const bf16x4*)(bias + n);
  bf16x4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = (bf16)(a[t] + (float)b4[t]);
  *(bf16x4*)(C + (int64_t)m * ldc + n) = r;
}

template <class G, int D, bool CONV = false>
void launch(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda, int ldb, int ldc,
            int splits, float* ws, hipStream_t s, Conv cv = {}) {
  // the ring, and the output staging (a TM x TN block per wave) inside it
  constexpr int LDS_BYTES = D * G::SLOT > G::WAVES * G::TM * G::RB ? D * G::SLOT : G::WAVES * G::TM * G::RB;
  static const bool attrs = [] {
    (void)hipFuncSetAttribute((const void*)gemm_f_kernel<G, D, CONV>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS_BYTES);
    return true;
  }();
  (void)attrs;
  const int tilesN = (N + G::BNT - 1) / G::BNT, tiles = ((M + BM - 1) / BM) * tilesN;
  hipLaunchKernelGGL((gemm_f_kernel<G, D, CONV>), dim3(tiles * splits), dim3(G::NT), LDS_BYTES, s,
                     (const bf16*)A, (const bf16*)B, (bf16*)C, (const bf16*)bias, M, N, K, lda, ldb, ldc, tilesN, cv,
                     splits, ws);
  if (splits > 1)
    hipLaunchKernelGGL(splitk_bias_kernel, dim3((unsigned)(((int64_t)M * N / 4 + 255) / 256)), dim3(256), 0, s, ws,
                       (const bf16*)bias, (bf16*)C, M, N, ldc, splits);
}

}  // namespace gemm_f
}  // namespace vcx

using namespace vcx;

bool vcx_gemm_f_supported(int M, int N, int K) {
  // N a multiple of 128 (a wave's columns are all in or all out), K a multiple of 64 and >= 192 (even slice
  // count, 3-deep ring), operand panels under 2 GB (32-bit buffer offsets)
  return M > 0 && N > 0 && (N % 128 == 0 || N == 64) && K % 64 == 0 && K >= 192 &&
         (int64_t)256 * K * 2 < (int64_t(1) << 31);
}

bool vcx_gemm_f_split_ok(int M, int N, int K, int splits) {
  const int nk = K / gemm_f::BKS;
  return splits >= 1 && splits <= 16 && nk % splits == 0 && (nk / splits) % 2 == 0 && nk / splits >= 6;
}

// K splits for an output of fewer tiles than CUs: the largest count that keeps splits x tiles within one round
// of 256 workgroups and each split's slice count even and >= 6 (1: no split)
int vcx_gemm_f_splits(int M, int N, int K) {
  const int bn = N <= 64 ? 64 : N <= 128 ? 128 : 256;  // the tile width vcx_gemm_f launches
  const int tiles = ((M + gemm_f::BM - 1) / gemm_f::BM) * ((N + bn - 1) / bn);
  int best = 1;
  for (int s = 2; s <= 16 && tiles * s <= 256; ++s)
    if (vcx_gemm_f_split_ok(M, N, K, s)) best = s;
  return best;
}

// waves: 4 (128 x 128 per wave) or 8 (128 x 64 per wave); anything else = the default (8); N = 128: 8 waves of
// 64 x 64 on a 256 x 128 tile; N = 64: 4 waves of 64 x 64 on a 256 x 64 tile. splits > 1: ws holds splits x M x N fp32 partials
void vcx_gemm_f(const void* A, const void* B, void* C, const void* bias, int M, int N, int K, int lda, int ldb,
                int ldc, int waves, int splits, float* ws, hipStream_t s) {
  if (N <= 64)  // the narrow tiles first: a 256-wide tile's waves store whole 64 / 128-column blocks
    gemm_f::launch<gemm_f::G4n, 4>(A, B, C, bias, M, N, K, lda, ldb, ldc, splits, ws, s);
  else if (N <= 128)
    gemm_f::launch<gemm_f::G8n, 4>(A, B, C, bias, M, N, K, lda, ldb, ldc, splits, ws, s);
  else if (waves == 4)
    gemm_f::launch<gemm_f::G4, 4>(A, B, C, bias, M, N, K, lda, ldb, ldc, splits, ws, s);
  else
    gemm_f::launch<gemm_f::G8, 4>(A, B, C, bias, M, N, K, lda, ldb, ldc, splits, ws, s);
}

static int log2_exact(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return (1 << l) == v ? l : -1;
}

bool vcx_gemm_f_conv3x3_supported(int imgs, int H, int W, int Cin, int Cout, int stride) {
  // Cin a power of two >= 64 (a 32-deep slice inside one tap, K = 9 Cin a multiple of 64), Cout a multiple of 128,
  // x under 2 GB (32-bit offsets), output rows in int
  const int lc = log2_exact(Cin);
  const int64_t Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  return imgs > 0 && H > 0 && W > 0 && lc >= 6 && (Cout % 128 == 0 || Cout == 64) && (stride == 1 || stride == 2) &&
         (int64_t)imgs * H * W * Cin * 2 < (int64_t(1) << 31) - (int64_t(1) << 20) && imgs * Ho * Wo < (int64_t(1) << 31) &&
         vcx_gemm_f_supported(1, Cout, 9 * Cin);
}

// y[imgs, Ho, Wo, Cout] (+ bias) = conv3x3(x[imgs, H, W, Cin], w[Cout][3][3][Cin]), pad 1; flip: the kernel's taps
// mirrored (w holds tap (ky, kx) where the convolution wants (2 - ky, 2 - kx): a stride-1 input gradient from the
// transposed weight without a flip copy); tap_major: w is [9][Cout][Cin] (each tap's [Cout][Cin] block in turn: the
// transpose of the channels-last weight matrix [Cin_conv, 9 Cout_conv], one transpose kernel)
void vcx_gemm_f_conv3x3(const void* x, const void* w, void* y, const void* bias, int imgs, int H, int W, int Cin,
                        int Cout, int stride, int waves, int splits, float* ws, int flip, int tap_major,
                        hipStream_t s) {
  gemm_f::Conv cv;
  cv.flip = flip;
  cv.btap = tap_major ? Cout * Cin : 0;
  cv.H = H;
  cv.W = W;
  cv.lc = log2_exact(Cin);
  cv.Ho = (H - 1) / stride + 1;
  cv.Wo = (W - 1) / stride + 1;
  cv.stride = stride;
  cv.xbytes = (unsigned)((int64_t)imgs * H * W * Cin * 2);
  const int M = imgs * cv.Ho * cv.Wo, K = 9 * Cin, ldb = tap_major ? Cin : K;
  if (Cout <= 64)
    gemm_f::launch<gemm_f::G4n, 4, true>(x, w, y, bias, M, Cout, K, 0, ldb, Cout, splits, ws, s, cv);
  else if (Cout <= 128)
    gemm_f::launch<gemm_f::G8n, 4, true>(x, w, y, bias, M, Cout, K, 0, ldb, Cout, splits, ws, s, cv);
  else if (waves == 4)
    gemm_f::launch<gemm_f::G4, 4, true>(x, w, y, bias, M, Cout, K, 0, ldb, Cout, splits, ws, s, cv);
  else
    gemm_f::launch<gemm_f::G8, 4, true>(x, w, y, bias, M, Cout, K, 0, ldb, Cout, splits, ws, s, cv);
}
