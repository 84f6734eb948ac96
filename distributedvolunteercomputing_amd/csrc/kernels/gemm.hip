// Hand-written bf16 MFMA GEMM for gfx950 with fused epilogues (GPT-2 MLP / projections).
//
//   C[M, N] = A[M, K] . B[N, K]^T        (both operands K-contiguous: x @ W^T, dY @ (W^T)^T)
//
// Why hand-written: hipBLASLt has no working bias+GELU / DGELU epilogue algorithms in this
// build, so the MLP paid two extra HBM passes per layer (bias_gelu_fwd, bias_gelu_bwd:
// 4.4 ms of a 62 ms GPT-2 step). This kernel writes the bias-added pre-activation AND the GELU
// output straight from the accumulators, and its backward variant multiplies the incoming
// gradient by gelu'(pre) and reduces the bias gradient (column sums) in the epilogue.
//
// Structure (CDNA4 playbook: cdna_hip_programming.md §5, T1/T2/T3/T4):
//   * 256 x 256 output tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 each),
//     v_mfma_f32_16x16x32_bf16, 128 fp32 accumulators per lane, one workgroup per CU.
//     (Measured alternative: 256 x 128 tiles with two 4-wave workgroups per CU, 3-slot rings —
//     20 % slower at the GPT-2 shapes.)
//   * operands staged HBM -> LDS with global_load_lds_dwordx4 (LDS-DMA: no staging VGPRs, no
//     ds_write), in a 4-slot ring of K-slices of 32 (32 KB per slot: A 256x32 + B 256x32).
//     Slice k+4 is issued into the slot of slice k while slice k is consumed from registers;
//     the wait for slice k+1 is a COUNTED s_waitcnt vmcnt(8) followed by a raw s_barrier, so
//     two slices stay in flight across every barrier (a __syncthreads() would drain them).
//   * fragments are double-buffered in registers: the ds_read_b128s of slice k+1 are issued
//     before the 32 MFMAs of slice k (even/odd unrolled, statically named register sets).
//   * LDS image: 64-B rows (32 bf16 of one slice), 16-B chunks XOR-swizzled by
//     F[(row >> 2) & 3] = {0,2,3,1}: every ds_read_b128 lane group (16 lanes: 16 rows, two
//     chunks) hits 16 distinct 16-B bank slots (conflict-free); LDS-DMA writes lane-linearly,
//     so the swizzle is applied to the per-lane GLOBAL source address (guide rule 21).
//   * operand order: mfma(W-fragment, X-fragment) so a lane's accumulator holds 4 consecutive
//     output COLUMNS of one row: row-contiguous 8-byte stores, per-column bias in registers.
//   * XCD-aware tile order (T1): blocks that share an XCD's L2 take consecutive tiles of the
//     same 256-row A panel.
#include <type_traits>

#include "vcx_common.h"

namespace vcx {
namespace gemm {

typedef short sx8 __attribute__((ext_vector_type(8)));

constexpr int BM = 256, BN = 256, BKS = 32, NSLOT = 4, NT = 512;
constexpr int ROWB = BKS * 2;                  // 64 bytes per row per slot
constexpr int SLOT_A = BM * ROWB;              // 16 KB
constexpr int SLOT_BYTES = (BM + BN) * ROWB;   // 32 KB
constexpr int LDS_BYTES = NSLOT * SLOT_BYTES;  // 128 KB

enum Epi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_DGELU = 3, EPI_BIAS_RELU = 4 };

// chunk swizzle F[(row >> 2) & 3] = {0, 2, 3, 1}, packed 2 bits per entry
__device__ __forceinline__ int swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

// s_waitcnt vmcnt(N) lgkmcnt(0) (N < 16; expcnt left at its maximum)
template <int N>
__device__ __forceinline__ void waitcnt() {
  static_assert(N >= 0 && N < 16, "vmcnt field");
  __builtin_amdgcn_s_waitcnt(0x0070 | N);
}
// raw barrier that the compiler may not move LDS reads across (the builtin is IntrNoMem)
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ void glds16(const bf16* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  // 0.5 x (1 + tanh(u)) = x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3)
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x * x, x);
  return x / (1.f + __expf(-u2));
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float x2 = x * x;
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x2, x);
  const float s = 1.f / (1.f + __expf(-u2));  // sigmoid(2u) = (1 + tanh u) / 2
  // d/dx [x s(2u)] = s + x s (1 - s) 2u',  2u' = sqrt(8/pi) (1 + 3 * 0.044715 x^2)
  return fmaf(x * s * (1.f - s), 1.5957691216057308f * fmaf(0.134145f, x2, 1.f), s);
}

struct Frags {
  sx8 x[8];  // X / A fragments: 8 row blocks of 16 (the wave's 128 rows of M)
  sx8 w[4];  // W / B fragments: 4 row blocks of 16 (the wave's 64 columns of N)
};

template <int EPI>
__global__ void __launch_bounds__(NT, 1)
    gemm_nt_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
                   bf16* __restrict__ C2, const bf16* __restrict__ bias, float* __restrict__ colsum, int M, int N,
                   int K, int lda, int ldb, int ldc, int tilesN) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  // ---- XCD-aware bijective tile order: consecutive logical tiles share an XCD (and its L2), and
  // the logical order walks GROUP_M row panels x all column panels in column-major blocks, so the
  // ~32 tiles an XCD runs at once are a 4 x 8 block (4 A + 8 B panels in flight) instead of one A
  // panel x 32 B panels (the whole B operand re-streamed by every XCD every round at large N)
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int wg = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + (bid >> 3);
  constexpr int GROUP_M = 4;
  const int tilesM = nwg / tilesN;
  const int per_group = GROUP_M * tilesN;
  const int gfirst = (wg / per_group) * GROUP_M;
  const int gsize = min(tilesM - gfirst, GROUP_M);
  const int m0 = (gfirst + (wg % per_group) % gsize) * BM, n0 = ((wg % per_group) / gsize) * BN;

  // ---- LDS-DMA staging: a slice is 32 pieces of 16 rows x 64 B (A: 16, B: 16); wave w moves
  // A pieces w, w+8 and B pieces w, w+8. Lane l of a piece writes LDS bytes [16 l, 16 l + 16):
  // row l >> 2, physical chunk l & 3, which holds logical chunk (l & 3) ^ swz(row) of that row
  const int prow = lane >> 2;
  const int pchunk = (lane & 3) ^ swz(prow);
  // ragged M (the detector's N*H*W rows): rows past M re-read row M - 1 (their outputs are never
  // stored), so no load leaves the operand
  const bf16* a_src = A + (int64_t)min(m0 + wid * 16 + prow, M - 1) * lda + pchunk * 8;
  const bf16* a_src8 = A + (int64_t)min(m0 + wid * 16 + prow + 128, M - 1) * lda + pchunk * 8;  // piece w + 8
  const bf16* b_src = B + (int64_t)(n0 + wid * 16 + prow) * ldb + pchunk * 8;
  const int64_t b_step8 = (int64_t)128 * ldb;
  char* const lds_piece = smem + wid * 1024;

  auto stage_piece = [&](int s, int p) {  // piece p (0..3: A w, A w+8, B w, B w+8) of K-slice s
    char* slot = lds_piece + (s & 3) * SLOT_BYTES;
    const int k0 = s * BKS;
    if (p == 0) glds16(a_src + k0, slot);
    if (p == 1) glds16(a_src8 + k0, slot + 8 * 1024);
    if (p == 2) glds16(b_src + k0, slot + SLOT_A);
    if (p == 3) glds16(b_src + b_step8 + k0, slot + SLOT_A + 8 * 1024);
  };
  auto stage = [&](int s) {
#pragma unroll
    for (int p = 0; p < 4; ++p) stage_piece(s, p);
  };

  // ---- fragment reads: lane l -> row (l & 15) of a 16-row block, k chunk (l >> 4)
  const int frow = lane & 15;
  const int foff = frow * ROWB + (((lane >> 4) ^ swz(frow)) << 4);
  const char* xa = smem + (wm * 128) * ROWB + foff;
  const char* wb = smem + SLOT_A + (wn * 64) * ROWB + foff;

  auto load_part = [&](Frags& f, int s, int part) {  // 0: x[0..3], 1: x[4..7], 2: w[0..3]
    const int so = (s & 3) * SLOT_BYTES;
    if (part < 2) {
#pragma unroll
      for (int i = 0; i < 4; ++i) f.x[4 * part + i] = *(const sx8*)(xa + so + (4 * part + i) * 16 * ROWB);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) f.w[j] = *(const sx8*)(wb + so + j * 16 * ROWB);
    }
  };
  auto load = [&](Frags& f, int s) {
#pragma unroll
    for (int part = 0; part < 3; ++part) load_part(f, s, part);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto mma = [&](const Frags& f, auto I0, auto I1) {  // row blocks [I0, I1) of the wave tile
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = decltype(I0)::value; i < decltype(I1)::value; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[j], f.x[i], acc[i][j], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  using I0c = std::integral_constant<int, 0>;
  using I2c = std::integral_constant<int, 2>;
  using I4c = std::integral_constant<int, 4>;
  using I6c = std::integral_constant<int, 6>;
  using I8c = std::integral_constant<int, 8>;

  const int nk = K / BKS;  // even and >= 4 (host checks K % 64 == 0, K >= 128)
  // Prefetch distance 4: step s issues slice s + 4 into the slot of slice s, whose fragments
  // are already in registers (read during step s - 1, retired by the lgkmcnt(0) before the
  // barrier). Two slices stay in flight across every barrier.
  stage(0);
  stage(1);
  stage(2);
  stage(3);
  waitcnt<12>();
  barrier();
  Frags f0, f1;
  load(f0, 0);

  // one step: slice s is in registers (fc); make slice s + 1 visible (counted vmcnt leaves the
  // slices behind it in flight), issue slice s + 4, read slice s + 1 into fn, MFMAs of slice s.
  // The 4 LDS-DMA pieces (~60 issue cycles each) and 12 ds_read_b128 are spread over the 4 MFMA
  // groups (8 MFMAs each), pinned by sched_barriers, instead of issued back to back after the
  // barrier where both waves of a SIMD would stall on them together. Compile-time flags keep
  // the loop body branch-free (a branch makes the compiler's LDS wait before the MFMAs an
  // lgkmcnt(0) that covers the prefetch).
  auto step = [&](int s, Frags& fc, Frags& fn, auto STAGE, auto LOAD, auto PEND) {
    constexpr bool st = decltype(STAGE)::value, ld = decltype(LOAD)::value;
    waitcnt<4 * decltype(PEND)::value>();  // own DMA of slice s + 1 retired; own ds_reads too
    barrier();  // ... everyone's; and nobody still reads the slot of slice s (now s + 4)
    if constexpr (st) stage_piece(s + 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I0c{}, I2c{});
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ld) load_part(fn, s + 1, 0);
    if constexpr (st) stage_piece(s + 4, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I2c{}, I4c{});
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ld) load_part(fn, s + 1, 1);
    if constexpr (st) stage_piece(s + 4, 2);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I4c{}, I6c{});
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ld) load_part(fn, s + 1, 2);
    if constexpr (st) stage_piece(s + 4, 3);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I6c{}, I8c{});
  };
  using T = std::true_type;
  using F = std::false_type;
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  int s = 0;
  for (; s + 5 < nk; s += 2) {  // steady state: slices up to s + 5 exist
    step(s, f0, f1, T{}, T{}, P2{});
    step(s + 1, f1, f0, T{}, T{}, P2{});
  }
  // s = nk - 4: nothing left to stage
  step(s, f0, f1, F{}, T{}, P2{});
  step(s + 1, f1, f0, F{}, T{}, P1{});
  step(s + 2, f0, f1, F{}, T{}, P0{});
  mma(f1, I0c{}, I8c{});

  // ---- epilogue: acc[i][j] holds C[m][n .. n+3], m = row block i, lane & 15; n = column block j
  const int mrow = m0 + wm * 128 + (lane & 15);
  const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
  float bsv[4][4];
  if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_RELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const bf16x4 bv = *(const bf16x4*)(bias + ncol + 16 * j);
#pragma unroll
      for (int t = 0; t < 4; ++t) bsv[j][t] = (float)bv[t];
    }
  }
  float cs[4][4];
  if constexpr (EPI == EPI_DGELU) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) cs[j][t] = 0.f;
  }
  // Output tiles leave through LDS: the accumulator layout gives each lane 8-B pieces of 16 rows
  // (a store instruction would touch 16 cache lines at 32 B each); staged per wave as a 128 x 64
  // bf16 block (16 KB, 16-B chunks XOR-swizzled by row: 2-way ds_write_b64, conflict-free
  // ds_read_b128), it is written back as full 128-B row segments, 16 B per lane. Measured: the
  // direct 8-B stores were a quarter of the kernel time at the GPT-2 shapes.
  __syncthreads();  // every wave is done with the operand ring (no LDS-DMA is in flight: vmcnt(0) above)
  char* const stg = smem + wid * 16384;
  auto stage_out = [&](int i, int j, bf16x4 v) {
    const int r = 16 * i + (lane & 15), c = 16 * j + 4 * (lane >> 4);
    *(bf16x4*)(stg + r * 128 + ((((c >> 3) ^ (r & 7))) << 4) + ((c >> 2) & 1) * 8) = v;
  };
  auto flush = [&](bf16* dst) {  // the wave's staged 128 x 64 block -> dst rows, 16 B per lane
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const int k = lane & 7;
    bf16* base = dst + (int64_t)(m0 + wm * 128) * ldc + n0 + wn * 64 + k * 8;
    const int mrem = M - (m0 + wm * 128);  // rows of this wave's block inside M
#pragma unroll
    for (int it = 0; it < 16; ++it) {
      const int r = it * 8 + (lane >> 3);
      const bf16x8 v = *(const bf16x8*)(stg + r * 128 + ((k ^ (r & 7)) << 4));
      if (r < mrem) *(bf16x8*)(base + (int64_t)r * ldc) = v;
    }
  };
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int64_t rowoff = (int64_t)(mrow + 16 * i) * ldc;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x4 out;
      if constexpr (EPI == EPI_STORE) {
#pragma unroll
        for (int t = 0; t < 4; ++t) out[t] = (bf16)acc[i][j][t];
      } else if constexpr (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int t = 0; t < 4; ++t) out[t] = (bf16)(acc[i][j][t] + bsv[j][t]);
      } else if constexpr (EPI == EPI_BIAS_RELU) {
#pragma unroll
        for (int t = 0; t < 4; ++t) out[t] = (bf16)fmaxf(acc[i][j][t] + bsv[j][t], 0.f);
      } else {  // EPI_DGELU: C2 holds the pre-activation, acc the gradient w.r.t. gelu(pre)
        const bf16x4 pre = *(const bf16x4*)(C2 + rowoff + ncol + 16 * j);
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const bf16 g = (bf16)(acc[i][j][t] * gelu_tanh_grad((float)pre[t]));
          out[t] = g;
          cs[j][t] += (float)g;
        }
      }
      stage_out(i, j, out);
    }
  }
  flush(C);
  if constexpr (EPI == EPI_BIAS_GELU) {  // second output: gelu(pre), through the same staging block
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        bf16x4 act;
#pragma unroll
        for (int t = 0; t < 4; ++t) act[t] = (bf16)gelu_tanh((float)(bf16)(acc[i][j][t] + bsv[j][t]));
        stage_out(i, j, act);
      }
    flush(C2);
  }
  if constexpr (EPI == EPI_DGELU) {
    // bias gradient: sum this wave's 128 rows per column (16 lanes share a column set), one
    // fp32 atomic per column per wave
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        float v = cs[j][t];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if ((lane & 15) == 0) atomicAdd(colsum + ncol + 16 * j + t, v);
      }
  }
}

// dst[r][c] = src[c][r] for a [R, Cc] bf16 matrix (weights: W -> W^T for the input-gradient GEMM)
__global__ void __launch_bounds__(256) transpose_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                             int R, int Cc) {
  __shared__ bf16 t[64][65];
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int rr = e >> 6, cc = e & 63;
    if (r0 + rr < R && c0 + cc < Cc) t[rr][cc] = src[(int64_t)(r0 + rr) * Cc + c0 + cc];
  }
  __syncthreads();
  for (int e = threadIdx.x; e < 64 * 64; e += 256) {
    const int cc = e >> 6, rr = e & 63;
    if (r0 + rr < R && c0 + cc < Cc) dst[(int64_t)(c0 + cc) * R + r0 + rr] = t[rr][cc];
  }
}

// the same with 16-B global loads and stores (R, Cc multiples of 8): each thread moves two 8-element
// row pieces into a padded LDS tile, then gathers two 8-element column pieces of it
__global__ void __launch_bounds__(256) transpose_bf16_v8_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                                int R, int Cc) {
  __shared__ __attribute__((aligned(16))) bf16 t[64][72];  // 144-B rows: 16-B aligned, reads spread over banks
  const int r0 = blockIdx.y * 64, c0 = blockIdx.x * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, rr = e >> 3, cc = (e & 7) * 8;
    if (r0 + rr < R && c0 + cc < Cc) *(bf16x8*)&t[rr][cc] = *(const bf16x8*)(src + (int64_t)(r0 + rr) * Cc + c0 + cc);
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int e = threadIdx.x + 256 * i, cc = e >> 3, rr = (e & 7) * 8;
    if (c0 + cc < Cc && r0 + rr < R) {
      bf16x8 v;
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = t[rr + j][cc];
      *(bf16x8*)(dst + (int64_t)(c0 + cc) * R + r0 + rr) = v;
    }
  }
}

// out_bf16[i] += (bf16) in_f32[i] (the epilogue's fp32 column sums into a flat .grad slot); zero_in: in[i] = 0
// afterwards (a zero-at-rest column-sum buffer: no fill launch before the next GEMM adds into it)
__global__ void __launch_bounds__(256) add_f32_into_bf16_kernel(float* __restrict__ in, bf16* __restrict__ out, int n,
                                                                int accumulate, int zero_in) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i < n) {
    out[i] = (bf16)((accumulate ? (float)out[i] : 0.f) + in[i]);
    if (zero_in) in[i] = 0.f;
  }
}

}  // namespace gemm
}  // namespace vcx

using namespace vcx;

bool vcx_gemm_nt_supported(int M, int N, int K) {
  return M > 0 && N > 0 && K >= 128 && M % gemm::BM == 0 && N % gemm::BN == 0 && K % 64 == 0;
}

// epilogues without a second operand read (STORE, BIAS, BIAS_RELU) also take a ragged M
bool vcx_gemm_nt_supported_epi(int M, int N, int K, int epi) {
  if (epi == gemm::EPI_STORE || epi == gemm::EPI_BIAS || epi == gemm::EPI_BIAS_RELU)
    return M > 0 && N > 0 && K >= 128 && N % gemm::BN == 0 && K % 64 == 0;
  return epi >= 0 && epi <= 3 && vcx_gemm_nt_supported(M, N, K);
}

// C = A . B^T with epilogue `epi` (gemm::Epi); colsum (EPI_DGELU) must be zeroed by the caller.
void vcx_gemm_nt(const void* A, const void* B, void* C, void* C2, const void* bias, float* colsum, int M, int N, int K,
                 int lda, int ldb, int ldc, int epi, hipStream_t s) {
  using namespace gemm;
  const int tilesN = N / BN, tiles = ((M + BM - 1) / BM) * tilesN;
  static const bool attrs = [] {  // 128 KB of dynamic LDS per workgroup (above the 64 KB default)
    for (const void* k : {(const void*)gemm_nt_kernel<EPI_STORE>, (const void*)gemm_nt_kernel<EPI_BIAS>,
                          (const void*)gemm_nt_kernel<EPI_BIAS_GELU>, (const void*)gemm_nt_kernel<EPI_DGELU>,
                          (const void*)gemm_nt_kernel<EPI_BIAS_RELU>})
      hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    return true;
  }();
  (void)attrs;
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tiles), dim3(NT), LDS_BYTES, s, (const bf16*)A, (const bf16*)B, (bf16*)C, (bf16*)C2,
                       (const bf16*)bias, colsum, M, N, K, lda, ldb, ldc, tilesN);
  };
  switch (epi) {
    case EPI_STORE: args(gemm_nt_kernel<EPI_STORE>); break;
    case EPI_BIAS: args(gemm_nt_kernel<EPI_BIAS>); break;
    case EPI_BIAS_GELU: args(gemm_nt_kernel<EPI_BIAS_GELU>); break;
    case EPI_BIAS_RELU: args(gemm_nt_kernel<EPI_BIAS_RELU>); break;
    default: args(gemm_nt_kernel<EPI_DGELU>); break;
  }
}

void vcx_transpose_bf16(const void* src, void* dst, int R, int Cc, hipStream_t s) {
  if (R % 8 == 0 && Cc % 8 == 0 && ((uintptr_t)src | (uintptr_t)dst) % 16 == 0) {
    hipLaunchKernelGGL(gemm::transpose_bf16_v8_kernel, dim3((Cc + 63) / 64, (R + 63) / 64), dim3(256), 0, s,
                       (const bf16*)src, (bf16*)dst, R, Cc);
    return;
  }
  hipLaunchKernelGGL(gemm::transpose_bf16_kernel, dim3((Cc + 63) / 64, (R + 63) / 64), dim3(256), 0, s,
                     (const bf16*)src, (bf16*)dst, R, Cc);
}

void vcx_add_f32_into_bf16(float* in, void* out, int n, int accumulate, int zero_in, hipStream_t s) {
  hipLaunchKernelGGL(gemm::add_f32_into_bf16_kernel, dim3((n + 255) / 256), dim3(256), 0, s, in, (bf16*)out, n,
                     accumulate, zero_in);
}
