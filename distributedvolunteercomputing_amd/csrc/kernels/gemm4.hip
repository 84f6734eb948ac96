// 4-wave, one-wave-per-SIMD bf16 MFMA GEMM for gfx950: C[M, N] = A[M, K] . B[N, K]^T.
//
// Why this decomposition (profiles/r3_gemm_persistent.txt): the 8-wave kernels of gemm.hip /
// gemm_persistent.hip put two waves on every SIMD, each with a 128 x 64 sub-tile; the two waves
// share the SIMD's MFMA pipe and every K-slice costs 12 LDS fragment reads per 32 MFMAs per wave.
// Here a 256-thread workgroup (one per CU, one wave per SIMD) computes the 256 x 256 tile as 2 x 2
// waves of 128 x 128: 256 fp32 accumulators per lane (the AGPR half of the 512-entry register
// file that a lone wave owns), 16 fragment reads per 64 MFMAs (a quarter fewer LDS bytes per
// MFMA), no pipe sharing, one barrier per 32-deep K-slice.
// Operands: HBM -> LDS by LDS-DMA (global_load_lds_dwordx4) into a 4-slot ring of 32-deep
// K-slices (32 KB per slot), counted s_waitcnt vmcnt + raw s_barrier (two slices in flight across
// every barrier), 16-B chunks XOR-swizzled (applied to the per-lane source address), A rows
// 0..6 single-buffered in registers and refilled right behind the MFMA row that used them, A row
// 7 and all B fragments double-buffered so every read of the next slice issues before the step's
// last MFMA row. Output tiles leave through the (then idle) ring as 256-B row segments.
// Reference analog: the compute hot loop /root/reference/worker.py:249.
#include <type_traits>

#include "vcx_common.h"

namespace vcx {
namespace gemm4 {

typedef short sx8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256, BN = 256, BKS = 32, NT = 256;
constexpr int ROWB = BKS * 2;           // 64 B per row of a slice image
constexpr int HALF = BM * ROWB;         // 16 KB
constexpr int SLOT = 2 * HALF;          // 32 KB
constexpr int LDS_BYTES = 4 * SLOT;     // 128 KB

__device__ __forceinline__ int swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  __builtin_amdgcn_s_waitcnt(0x0070 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ void glds16(const bf16* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__global__ void __launch_bounds__(NT, 1)
    gemm4_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C, int M, int N, int K,
                 int lda, int ldb, int ldc, int tilesN) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 1, wn = wid & 1;

  // XCD-aware bijective tile order, GROUP_M row panels x all column panels per group
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GROUP_M = 4;
  const int tilesM = nwg / tilesN;
  const int per_group = GROUP_M * tilesN;
  const int gfirst = (wg / per_group) * GROUP_M;
  const int gsize = min(tilesM - gfirst, GROUP_M);
  const int m0 = (gfirst + (wg % per_group) % gsize) * BM, n0 = ((wg % per_group) / gsize) * BN;

  // staging: a slice = 16 A pieces + 16 B pieces of 16 rows x 64 B; wave w moves pieces w + 4j
  const int prow = lane >> 2;
  const int pch = ((lane & 3) ^ swz(prow)) * 8;
  const bf16* a_src = A + (int64_t)(m0 + wid * 16 + prow) * lda + pch;
  const bf16* b_src = B + (int64_t)(n0 + wid * 16 + prow) * ldb + pch;
  const int64_t a64 = (int64_t)64 * lda, b64 = (int64_t)64 * ldb;
  auto stage_piece = [&](char* slotp, int s, auto P) {
    constexpr int p = decltype(P)::value, j = p & 3;
    const int k0 = s * BKS;
    if constexpr (p < 4)
      glds16(a_src + j * a64 + k0, slotp + (wid + 4 * j) * 1024);
    else
      glds16(b_src + j * b64 + k0, slotp + HALF + (wid + 4 * j) * 1024);
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;
  using P4 = std::integral_constant<int, 4>;
  using P5 = std::integral_constant<int, 5>;
  using P6 = std::integral_constant<int, 6>;
  using P7 = std::integral_constant<int, 7>;
  auto stage_all = [&](char* slotp, int s) {
    stage_piece(slotp, s, P0{}), stage_piece(slotp, s, P1{}), stage_piece(slotp, s, P2{}),
        stage_piece(slotp, s, P3{}), stage_piece(slotp, s, P4{}), stage_piece(slotp, s, P5{}),
        stage_piece(slotp, s, P6{}), stage_piece(slotp, s, P7{});
  };

  // fragments: lane l -> row (l & 15) of a 16-row block, k chunk (l >> 4)
  const int frow = lane & 15;
  const int foff = frow * ROWB + (((lane >> 4) ^ swz(frow)) << 4);
  const int xo = (wm * 128) * ROWB + foff;
  const int wo = HALF + (wn * 128) * ROWB + foff;
  sx8 x[7], yA, yB, wA[8], wB[8];
  auto ld_x = [&](int so, int i) -> sx8 { return *(const sx8*)(smem + so + xo + i * 16 * ROWB); };
  auto ld_w = [&](sx8(&w)[8], int so) {
#pragma unroll
    for (int j = 0; j < 8; ++j) w[j] = *(const sx8*)(smem + so + wo + j * 16 * ROWB);
  };

  f32x4 acc[8][8];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto row = [&](const sx8& xf, const sx8(&w)[8], int i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xf, acc[i][j], 0, 0, 0);
  };

  const int nk = K / BKS;  // even, >= 4
  // one step: slice s in registers (x, yc, wc); loads of slice s + 1 interleaved with the 8 MFMA
  // rows; the 8 DMA pieces of slice s + 4 go into slice s's slot (read in step s - 1)
  auto step = [&](int s, sx8& yc, sx8(&wc)[8], sx8& yn, sx8(&wn)[8], auto ST, auto PEND) {
    constexpr bool st = decltype(ST)::value;
    wait_vm<decltype(PEND)::value>();
    barrier();
    char* slotp = smem + (s & 3) * SLOT;
    const int so = ((s + 1) & 3) * SLOT;
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (i < 7)
        row(x[i < 7 ? i : 0], wc, i);
      else
        row(yc, wc, 7);
      __builtin_amdgcn_sched_barrier(0);
      if (i < 7) x[i < 7 ? i : 0] = ld_x(so, i);
      if (i == 0) ld_w(wn, so);
      if (i == 1) yn = ld_x(so, 7);
      if constexpr (st) {
        if (i == 0) stage_piece(slotp, s + 4, P0{}), stage_piece(slotp, s + 4, P4{});
        if (i == 2) stage_piece(slotp, s + 4, P1{}), stage_piece(slotp, s + 4, P5{});
        if (i == 4) stage_piece(slotp, s + 4, P2{}), stage_piece(slotp, s + 4, P6{});
        if (i == 5) stage_piece(slotp, s + 4, P3{}), stage_piece(slotp, s + 4, P7{});
      }
      __builtin_amdgcn_sched_barrier(0);
    }
    __builtin_amdgcn_s_setprio(0);
  };
  using T = std::true_type;
  using F = std::false_type;
  using V16 = std::integral_constant<int, 16>;
  using V8 = std::integral_constant<int, 8>;
  using V0 = std::integral_constant<int, 0>;

  stage_all(smem, 0);
  stage_all(smem + SLOT, 1);
  stage_all(smem + 2 * SLOT, 2);
  stage_all(smem + 3 * SLOT, 3);
  wait_vm<24>();
  barrier();
#pragma unroll
  for (int i = 0; i < 7; ++i) x[i] = ld_x(0, i);
  yA = ld_x(0, 7);
  ld_w(wA, 0);
  int s = 0;
  for (; s + 5 < nk; s += 2) {
    step(s, yA, wA, yB, wB, T{}, V16{});
    step(s + 1, yB, wB, yA, wA, T{}, V16{});
  }
  step(s, yA, wA, yB, wB, F{}, V16{});
  step(s + 1, yB, wB, yA, wA, F{}, V8{});
  step(s + 2, yA, wA, yB, wB, F{}, V0{});
  // last slice: no more loads
  __builtin_amdgcn_s_waitcnt(0xC07F);
  barrier();
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 7; ++i) row(x[i], wB, i);
  row(yB, wB, 7);
  __builtin_amdgcn_s_setprio(0);

  // epilogue: each wave stages its 128 x 128 bf16 block (32 KB, the ring is idle now) in 128 x
  // 256-B rows, 16-B chunks XOR-swizzled by (row & 15), and writes 256-B row segments, 16 B / lane
  barrier();  // every wave is done reading the ring
  char* stg = smem + wid * 32768;
  const int cl = 4 * (lane >> 4);
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      bf16x4 o;
#pragma unroll
      for (int t = 0; t < 4; ++t) o[t] = (bf16)acc[i][j][t];
      const int rr = 16 * i + frow, c = 16 * j + cl;
      *(bf16x4*)(stg + rr * 256 + ((((c >> 3) ^ (rr & 15))) << 4) + ((c >> 2) & 1) * 8) = o;
    }
  __builtin_amdgcn_s_waitcnt(0xC07F);
  const int k16 = lane & 15, rl = lane >> 4;
  bf16* base = C + (int64_t)(m0 + wm * 128) * ldc + n0 + wn * 128 + k16 * 8;
#pragma unroll
  for (int it = 0; it < 32; ++it) {
    const int rr = it * 4 + rl;
    const bf16x8 v = *(const bf16x8*)(stg + rr * 256 + ((k16 ^ (rr & 15)) << 4));
    *(bf16x8*)(base + (int64_t)rr * ldc) = v;
  }
}

}  // namespace gemm4
}  // namespace vcx

using namespace vcx;

bool vcx_gemm4_supported(int M, int N, int K) {
  return M > 0 && N > 0 && M % gemm4::BM == 0 && N % gemm4::BN == 0 && K % 64 == 0 && K >= 128;
}

void vcx_gemm4(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc, hipStream_t s) {
  using namespace gemm4;
  static const bool attrs = [] {
    (void)hipFuncSetAttribute((const void*)gemm4_kernel, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    return true;
  }();
  (void)attrs;
  const int tilesN = N / BN, tiles = (M / BM) * tilesN;
  hipLaunchKernelGGL(gemm4_kernel, dim3(tiles), dim3(NT), LDS_BYTES, s, (const bf16*)A, (const bf16*)B, (bf16*)C, M,
                     N, K, lda, ldb, ldc, tilesN);
}
