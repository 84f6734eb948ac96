// Persistent, store-overlapped bf16 MFMA GEMM for gfx950:  C[M, N] = A[M, K] . B[N, K]^T
// with STORE / BIAS / BIAS+GELU epilogues (the GPT-2 forward projections and the MLP's fc).
//
// Why (profiles/r3_gemm_persistent.txt, r3_gemm_ps.txt): at the GPT-2 token-major shapes
// (M = 65536, K = 768) every 256 x 256 tile runs only 24 K-slices, and the per-tile prologue
// (first operand slices in flight from HBM) plus the epilogue (128 KB of output per tile, written
// while the CU's MFMA pipes idle) cost the tiled kernels -- ours and the library's -- 25-35 % of
// the main-loop rate. Here one 512-thread workgroup per CU walks its tiles with:
//   * the main loop of gemm_nt (gemm.hip): 8 waves as 2 (M) x 4 (N), 128 x 64 per wave,
//     v_mfma_f32_16x16x32_bf16, a 4-slot LDS-DMA ring of 32-deep K-slices, counted vmcnt + raw
//     s_barrier, fragments double-buffered in registers, LDS-DMA pieces and ds_reads interleaved
//     between the MFMA groups;
//   * ONE continuous ring across tile boundaries: the last 4 steps of tile t stage slices 0..3
//     of tile t + 1, so the next tile's first MFMAs never wait on a cold HBM round trip;
//   * an epilogue that needs neither LDS nor a barrier: v_permlane16_swap pairs two 16 x 16
//     accumulator blocks so that every lane holds 8 consecutive output columns (16-B stores, 64-B
//     row segments per 4 lanes). The stores are issued once the next tile's slices 0..3 have
//     landed and drain while that tile's first steps compute: its steps 0..2 need no vmcnt wait,
//     and the first counted wait (step 3) is for a slice issued after the stores. (Stores were
//     measured to retire ahead of older LDS-DMA on vmcnt, so a count that leaves stores in flight
//     across a wait for older DMA is not safe.)
//   * buffer resources per tile (uniform bases in SGPRs, tile-invariant per-lane offsets), and
//     the bias row resident in LDS (read once per workgroup).
// Tile walk: tile vb = blockIdx.x + k * gridDim.x through the bijective XCD-aware remap of
// gemm.hip (grouped 4 x 8 row/column panel blocks per XCD).
// Reference analog: the compute hot loop /root/reference/worker.py:249.
#include <type_traits>

#include "vcx_common.h"

namespace vcx {
namespace gemm_ps {

typedef short sx8 __attribute__((ext_vector_type(8)));
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BN = 256, BKS = 32, NT = 512;
constexpr int ROWB = BKS * 2;           // 64 B per row per slot
constexpr int SLOT_A = BM * ROWB;       // 16 KB
constexpr int SLOT = 2 * SLOT_A;        // 32 KB
constexpr int RING = 4 * SLOT;          // 128 KB
constexpr int BIAS_MAX = 16384;         // bias row resident in LDS behind the ring (32 KB)

// (3 is not used: gemm_nt's code 3 is DGELU, so a caller reusing its numbering is refused)
// EPI_BIAS_GELU_D (round 6): the fc forward writes gelu'(pre) to C instead of pre (and gelu(pre) to C2):
// pre is read by nothing but the backward's gelu', so the forward, which already has sigmoid(2u) for gelu,
// finishes gelu' in 4 more VALU ops per element, and the fc2 input gradient's epilogue (EPI_DMUL) is one
// multiply instead of the ~16 VALU ops + 2 transcendentals of gelu'(pre) (EPI_DGELU ran at 29 % MFMA busy,
// 473 vs 286 us for the same GEMM without an epilogue, profiles/r6_gpt2_step_pmc.txt).
enum Epi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_DGELU = 4, EPI_BIAS_GELU_D = 5, EPI_DMUL = 6 };
template <int E>
constexpr bool has_bias() { return E == EPI_BIAS || E == EPI_BIAS_GELU || E == EPI_BIAS_GELU_D; }
template <int E>
constexpr bool reads_c2() { return E == EPI_DGELU || E == EPI_DMUL; }

__device__ __forceinline__ int swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }

// s_waitcnt vmcnt(N) lgkmcnt(0) (N < 64; expcnt left at its maximum)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  __builtin_amdgcn_s_waitcnt(0x0070 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float x2 = x * x;
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x2, x);
  const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-u2));  // sigmoid(2u) = (1 + tanh u) / 2
  // d/dx [x sigmoid(2u)] = s + x s (1 - s) 2u',  2u' = sqrt(8/pi) (1 + 3 * 0.044715 x^2)
  return fmaf(x * sg * (1.f - sg), 1.5957691216057308f * fmaf(0.134145f, x2, 1.f), sg);
}

// gelu(x) and gelu'(x) sharing sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3)
__device__ __forceinline__ void gelu_and_grad(float x, float& act, float& grad) {
  const float x2 = x * x;
  const float u2 = x * fmaf(1.5957691216057308f * 0.044715f, x2, 1.5957691216057308f);
  const float sg = __builtin_amdgcn_rcpf(1.f + __expf(-u2));
  act = x * sg;
  grad = fmaf(act * (1.f - sg), fmaf(1.5957691216057308f * 0.134145f, x2, 1.5957691216057308f), sg);
}

__device__ __forceinline__ float gelu_tanh(float x) {
  // x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3); hardware reciprocal (the IEEE divide was
  // a 10-instruction v_div_scale/fmas/fixup sequence per element)
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x * x, x);
  return x * __builtin_amdgcn_rcpf(1.f + __expf(-u2));
}

// 16-B non-temporal buffer store as inline asm ending in `s_nop 1`: hipcc let a VALU write overwrite
// the data VGPRs of a builtin buffer_store_dwordx4 4 instructions after it (lanes 12-15 of each row
// stored stale dword 1, measured), so the store's read of its data registers is padded by hand
// (cdna_hip_programming.md §5.7 item 1, stores). nt: the GPT-2 shapes ran 7-14 % faster than with
// plain stores (profiles/r4_gemm_ps_diag.txt).
__device__ __forceinline__ void store16(u32x4 v, u32x4 desc, int voff, int soff) {
  asm volatile("buffer_store_dwordx4 %0, %1, %2, %3 offen nt\n\ts_nop 1" ::"v"(v), "v"(voff), "s"(desc), "s"(soff)
               : "memory");
}

// raw buffer descriptor words: 48-bit base, stride 0, num_records bytes, the flags word used by
// __builtin_amdgcn_make_buffer_rsrc elsewhere in the tree
__device__ __forceinline__ u32x4 desc_of(const void* base, int bytes) {
  const uint64_t a = (uint64_t)base;
  return u32x4{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, (unsigned)bytes, 0x00020000u};
}

// Workgroup geometry: one 512-thread workgroup (8 waves) per CU, 256 x 256 tiles, a 4-slot ring
struct Geo {
  static constexpr int NW = 8, NTH = NW * 64, BNt = 256, WNC = NW / 2, NSLOT = 4;
  static constexpr int SLOTA = BM * ROWB, SLOTB = SLOTA + BNt * ROWB, RINGB = NSLOT * SLOTB;
  static constexpr int APW = 16 / NW, BPW = BNt / 16 / NW, PPW = APW + BPW;  // LDS-DMA pieces per wave
  static constexpr int VMW = PPW * (NSLOT - 2);  // vmcnt of a step: the slices younger than the awaited one
};

struct Frags {
  sx8 y[2];  // A fragments of the wave's row blocks 6, 7
  sx8 w[4];  // B fragments: the wave's 4 column blocks of 16
};

template <int EPI>
__global__ void __launch_bounds__(512, 1)
    gemm_ps_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
                   bf16* __restrict__ C2, const bf16* __restrict__ bias, float* __restrict__ colsum, int M, int N,
                   int K, int lda, int ldb, int ldc, int tilesN, int tiles) {
  using Gm = Geo;
  constexpr int NW = Gm::NW, BNt = Gm::BNt, SLOTA = Gm::SLOTA, SLOTB = Gm::SLOTB, RINGB = Gm::RINGB,
                NSLOT = Gm::NSLOT;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid / Gm::WNC, wn = wid % Gm::WNC;
  const int G = gridDim.x, bid = blockIdx.x;
  const int nk = K / BKS;  // multiple of 4, >= 8 (host check)

  if constexpr (has_bias<EPI>()) {  // the bias row, once per workgroup
    bf16* bl = (bf16*)(smem + RINGB);
    for (int c = tid * 8; c < N; c += Gm::NTH * 8) *(bf16x8*)(bl + c) = *(const bf16x8*)(bias + c);
    __syncthreads();
  }

  // ---- tile coordinates: XCD-aware bijective remap (G is a multiple of 8 or equals tiles)
  const int q8 = tiles >> 3, r8 = tiles & 7;
  constexpr int GROUP_M = 4;
  const int tilesM = tiles / tilesN;
  auto coords = [&](int vb, int& m0, int& n0) {
    const int xcd = vb & 7;
    const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (vb >> 3);
    const int per_group = GROUP_M * tilesN;
    const int gfirst = (wg / per_group) * GROUP_M;
    const int gsize = min(tilesM - gfirst, GROUP_M);
    const int rr = wg - (wg / per_group) * per_group;
    m0 = (gfirst + rr % gsize) * BM;
    n0 = (rr / gsize) * BNt;
  };

  // ---- LDS-DMA staging through per-tile buffer resources; per-lane offsets are tile-invariant.
  // A slice is 32 pieces of 16 rows x 64 B (A: 16, B: 16); wave w moves A pieces w, w + 8 and B
  // pieces w, w + 8; lane l writes LDS bytes [16 l, 16 l + 16) of a piece: row l >> 2, physical
  // chunk l & 3 holding logical chunk (l & 3) ^ swz(row) (swizzle applied to the source address)
  const int prow = lane >> 2;
  const int pch = (lane & 3) ^ swz(prow);
  // piece p < APW: A rows (wid + NW p) * 16 + prow; else B rows (wid + NW (p - APW)) * 16 + prow
  const int a_off0 = ((wid * 16 + prow) * lda + pch * 8) * 2, a_pstep = NW * 16 * lda * 2;
  const int b_off0 = ((wid * 16 + prow) * ldb + pch * 8) * 2, b_pstep = NW * 16 * ldb * 2;
  char* const lds_piece = smem + wid * 1024;
  auto rsrc = [](const bf16* base, int bytes) {
    return __builtin_amdgcn_make_buffer_rsrc((void*)base, (short)0, bytes, 0x00020000);
  };
  using Rs = __amdgpu_buffer_rsrc_t;  // (decltype of the builtin call made the host pass drop the kernel stubs)
  auto tile_rs = [&](int vb, Rs& ra, Rs& rb) {
    int m0, n0;
    coords(vb, m0, n0);
    ra = rsrc(A + (int64_t)m0 * lda, BM * lda * 2);
    rb = rsrc(B + (int64_t)n0 * ldb, BNt * ldb * 2);
  };
  auto stage_piece = [&](const Rs& ra, const Rs& rb, int kslice, int slot, auto P) {
    constexpr int p = decltype(P)::value;
    char* sl = lds_piece + slot * SLOTB;
    const int soff = kslice * (BKS * 2);
    if constexpr (p < Gm::APW)
      __builtin_amdgcn_raw_ptr_buffer_load_lds(ra, (__attribute__((address_space(3))) void*)(sl + NW * p * 1024), 16,
                                               a_off0 + p * a_pstep, soff, 0, 0);
    else
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          rb, (__attribute__((address_space(3))) void*)(sl + SLOTA + NW * (p - Gm::APW) * 1024), 16,
          b_off0 + (p - Gm::APW) * b_pstep, soff, 0, 0);
  };
  // the 4 pieces of one slice, one per MFMA group of the step
  auto stage_group = [&](const Rs& ra, const Rs& rb, int kslice, int slot, auto GR) {
    static_assert(Gm::PPW == 4, "pieces per wave");
    stage_piece(ra, rb, kslice, slot, std::integral_constant<int, decltype(GR)::value>{});
  };
  using P0 = std::integral_constant<int, 0>;
  using P1 = std::integral_constant<int, 1>;
  using P2 = std::integral_constant<int, 2>;
  using P3 = std::integral_constant<int, 3>;

  // ---- fragment reads: lane l -> row (l & 15) of a 16-row block, k chunk (l >> 4)
  const int frow = lane & 15;
  const int foff = frow * ROWB + (((lane >> 4) ^ swz(frow)) << 4);
  const char* xa = smem + (wm * 128) * ROWB + foff;
  const char* wb = smem + SLOTA + (wn * 64) * ROWB + foff;
  // A rows 0..5 are single-buffered (x, refilled right behind the MFMA group that used them);
  // rows 6, 7 and the B fragments alternate between two named sets (Frags), so every read of the
  // next slice is issued before the step's last MFMA group (96 -> 72 fragment VGPRs)
  sx8 x[6];
  auto load_x = [&](int slot, int i0) {
    const int so = slot * SLOTB;
    x[i0] = *(const sx8*)(xa + so + i0 * 16 * ROWB);
    x[i0 + 1] = *(const sx8*)(xa + so + (i0 + 1) * 16 * ROWB);
  };
  auto load_w = [&](Frags& f, int slot, int j0) {
    const int so = slot * SLOTB;
    f.w[j0] = *(const sx8*)(wb + so + j0 * 16 * ROWB);
    f.w[j0 + 1] = *(const sx8*)(wb + so + (j0 + 1) * 16 * ROWB);
  };
  auto load_y = [&](Frags& f, int slot) {
    const int so = slot * SLOTB;
    f.y[0] = *(const sx8*)(xa + so + 6 * 16 * ROWB);
    f.y[1] = *(const sx8*)(xa + so + 7 * 16 * ROWB);
  };

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  auto mma = [&](const Frags& f, auto I0, auto I1) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = decltype(I0)::value; i < decltype(I1)::value; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const sx8& xf = i < 6 ? x[i < 6 ? i : 0] : f.y[i >= 6 ? i - 6 : 0];
        // in-place accumulation pinned by the "+v" constraint (the builtin let the register allocator
        // rotate accumulators between MFMAs, 174 of 384 not in place, and spill). An accumulate chain
        // needs no wait states; the epilogue's readers of acc are padded below.
        asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+v"(acc[i][j]) : "v"(f.w[j]), "v"(xf));
      }
    __builtin_amdgcn_s_setprio(0);
  };
  using I0c = std::integral_constant<int, 0>;
  using I2c = std::integral_constant<int, 2>;
  using I4c = std::integral_constant<int, 4>;
  using I6c = std::integral_constant<int, 6>;
  using I8c = std::integral_constant<int, 8>;

  // one step: slice s (slot s & 3) is in registers (x, fc); wait for slice s + 1, stage slice
  // s + 4 into slot s & 3 (the next tile's slice s + 4 - nk in the tile's last 4 steps), MFMAs of
  // slice s interleaved with the staging pieces and the fragment reads of slice s + 1 into (x, fn).
  // The wait: slices 0..3 of a tile all landed before the previous tile's epilogue issued its
  // stores (vmcnt(0) there), so steps 0..2 only retire their LDS reads; from step 3 on the awaited
  // slice was issued after those stores, and vmcnt(8) (slices s + 2, s + 3 in flight) also waits
  // for the stores. (Counting stores as younger ops in flight is not safe: stores retired ahead
  // of older operand DMA on vmcnt, measured as rare wrong tiles.)
  auto step = [&](int s, Frags& fc, Frags& fn, const Rs& sa, const Rs& sb, int ks, bool nowait, auto LD,
                  auto VM, auto ST) {
    constexpr bool ld = decltype(LD)::value, st = decltype(ST)::value;
    if (nowait)
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    else
      wait_vm<decltype(VM)::value>();
    barrier();
    const int slot = s % NSLOT, nslot = (s + 1) % NSLOT;
    if constexpr (st) stage_group(sa, sb, ks, slot, P0{});
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I0c{}, I2c{});
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ld) load_x(nslot, 0), load_w(fn, nslot, 0);
    if constexpr (st) stage_group(sa, sb, ks, slot, P1{});
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I2c{}, I4c{});
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ld) load_x(nslot, 2), load_w(fn, nslot, 2);
    if constexpr (st) stage_group(sa, sb, ks, slot, P2{});
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I4c{}, I6c{});
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (ld) load_x(nslot, 4), load_y(fn, nslot);
    if constexpr (st) stage_group(sa, sb, ks, slot, P3{});
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I6c{}, I8c{});
  };

  // ---- epilogue: acc[i][j] holds C[row 16 i + (l & 15)][col 16 j + 4 (l >> 4) + t]. One
  // v_permlane16_swap per accumulator register pairs column blocks (2 jp, 2 jp + 1): afterwards
  // lane group g holds 8 consecutive columns 16 (2 jp + (g & 1)) + 8 (g >> 1) of its row.
  const int g = lane >> 4;
  const int ccol = wn * 64 + 16 * (g & 1) + 8 * (g >> 1);  // + 32 jp
  // store A of row block i: lanes of rows 0..7 write (row r, jp 0), rows 8..15 write (row r - 8,
  // jp 1); store B is 8 rows further down
  const int c_offA = ((wm * 128 + (frow & 7)) * ldc + ccol + ((frow & 8) ? 32 : 0)) * 2;
  const bf16* bl = (const bf16*)(smem + RINGB);
  // EPI_DGELU: the pre-activation tile, read into registers (16 KB per wave) while the tile's last
  // step computes, at the positions the exchanged stores write
  u32x4 pre[8][2];
  auto load_pre = [&](int m0, int n0) {
    const Rs rp = rsrc(C2 + (int64_t)m0 * ldc + n0, BM * ldc * 2);
#pragma unroll
    for (int i = 0; i < 8; ++i)
#pragma unroll
      for (int q = 0; q < 2; ++q)
        pre[i][q] = __builtin_bit_cast(u32x4, __builtin_amdgcn_raw_buffer_load_b128(rp, c_offA + q * 8 * ldc * 2,
                                                                                      i * 16 * ldc * 2, 0));
  };
  auto epilogue = [&](int m0, int n0, auto DRAIN) {
    float cs[8];  // EPI_DGELU: fp32 column sums of this lane's 8 columns over its 16 rows
#pragma unroll
    for (int e = 0; e < 8; ++e) cs[e] = 0.f;
    // the next tile's slices 0..3 land before any store is issued (see step); the last MFMAs'
    // results -> VALU readers (v_permlane16_swap): 12 wait states for an 8-pass XDL op; the MFMAs are
    // inline asm, so hipcc's hazard recognizer does not pad this
    if constexpr (decltype(DRAIN)::value)
      asm volatile("s_waitcnt vmcnt(0)\n\ts_nop 7\n\ts_nop 4" ::: "memory");
    else
      asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const u32x4 rc = desc_of(C + (int64_t)m0 * ldc + n0, BM * ldc * 2);
    u32x4 rc2;
    if constexpr (EPI == EPI_BIAS_GELU || EPI == EPI_BIAS_GELU_D) rc2 = desc_of(C2 + (int64_t)m0 * ldc + n0, BM * ldc * 2);
    float bv[2][8];
    if constexpr (has_bias<EPI>()) {
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const bf16x8 b8 = *(const bf16x8*)(bl + n0 + ccol + 32 * jp);
#pragma unroll
        for (int e = 0; e < 8; ++e) bv[jp][e] = (float)b8[e];
      }
    }
    const bool lo = (lane & 8) == 0;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int soff = i * 16 * ldc * 2;
      u32x4 v[2];
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        float o[8];
#pragma unroll
        for (int t = 0; t < 4; ++t) {
          const u32x2 r = __builtin_amdgcn_permlane16_swap(__float_as_uint(acc[i][2 * jp][t]),
                                                          __float_as_uint(acc[i][2 * jp + 1][t]), false, false);
          o[t] = __uint_as_float(r.x);
          o[4 + t] = __uint_as_float(r.y);
        }
        acc[i][2 * jp] = f32x4{0.f, 0.f, 0.f, 0.f};
        acc[i][2 * jp + 1] = f32x4{0.f, 0.f, 0.f, 0.f};
        bf16x8 h;
#pragma unroll
        for (int e = 0; e < 8; ++e) h[e] = (bf16)(has_bias<EPI>() ? o[e] + bv[jp][e] : o[e]);
        v[jp] = __builtin_bit_cast(u32x4, h);
      }
      // rows r and r ^ 8 of the 16-row block trade halves (DPP row_ror:8): lanes of rows 0..7 keep
      // their jp = 0 chunk and take row r + 8's; rows 8..15 keep jp = 1 and take row r - 8's. Store
      // A then writes rows 0..7 and store B rows 8..15, each as 8 full 128-B row segments.
#pragma unroll
      for (int d = 0; d < 4; ++d) {
        const int x = (int)(lo ? v[1][d] : v[0][d]);
        const unsigned y = (unsigned)__builtin_amdgcn_update_dpp(0, x, 0x128, 0xF, 0xF, false);
        if (lo)
          v[1][d] = y;
        else
          v[0][d] = y;
      }
      if constexpr (EPI == EPI_DMUL) {  // v = dY W (the gradient w.r.t. gelu(pre)), gelu'(pre) from registers
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bf16x8 g8 = __builtin_bit_cast(bf16x8, v[q]), p8 = __builtin_bit_cast(bf16x8, pre[i][q]);
          bf16x8 o8;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = (float)g8[e] * (float)p8[e];
            cs[e] += d;
            o8[e] = (bf16)d;
          }
          v[q] = __builtin_bit_cast(u32x4, o8);
        }
      }
      if constexpr (EPI == EPI_BIAS_GELU_D) {  // v = pre (bf16): C gets gelu'(pre), C2 gelu(pre)
        u32x4 av[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bf16x8 p8 = __builtin_bit_cast(bf16x8, v[q]);
          bf16x8 a8, g8;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float a, g;
            gelu_and_grad((float)p8[e], a, g);
            a8[e] = (bf16)a;
            g8[e] = (bf16)g;
          }
          v[q] = __builtin_bit_cast(u32x4, g8);
          av[q] = __builtin_bit_cast(u32x4, a8);
        }
        store16(v[0], rc, c_offA, soff);
        store16(v[1], rc, c_offA + 8 * ldc * 2, soff);
        store16(av[0], rc2, c_offA, soff);
        store16(av[1], rc2, c_offA + 8 * ldc * 2, soff);
        continue;
      }
      if constexpr (EPI == EPI_DGELU) {  // v = dY W (the gradient w.r.t. gelu(pre)), pre from registers
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bf16x8 g8 = __builtin_bit_cast(bf16x8, v[q]), p8 = __builtin_bit_cast(bf16x8, pre[i][q]);
          bf16x8 o8;
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            const float d = (float)g8[e] * gelu_tanh_grad((float)p8[e]);
            cs[e] += d;
            o8[e] = (bf16)d;
          }
          v[q] = __builtin_bit_cast(u32x4, o8);
        }
      }
      store16(v[0], rc, c_offA, soff);
      store16(v[1], rc, c_offA + 8 * ldc * 2, soff);
      if constexpr (EPI == EPI_BIAS_GELU) {
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const bf16x8 pre = __builtin_bit_cast(bf16x8, v[q]);
          bf16x8 act;
#pragma unroll
          for (int e = 0; e < 8; ++e) act[e] = (bf16)gelu_tanh((float)pre[e]);
          store16(__builtin_bit_cast(u32x4, act), rc2, c_offA + q * 8 * ldc * 2, soff);
        }
      }
    }
    if constexpr (reads_c2<EPI>()) {
      // bias gradient: the 8 lanes of rows 0..7 (lane bits 0..2) share the same 8 columns
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float t = cs[e];
        t += __shfl_xor(t, 1, 64);
        t += __shfl_xor(t, 2, 64);
        t += __shfl_xor(t, 4, 64);
        cs[e] = t;
      }
      if ((lane & 7) == 0) {
        float* dst = colsum + n0 + ccol + ((frow & 8) ? 32 : 0);
#pragma unroll
        for (int e = 0; e < 8; ++e) atomicAdd(dst + e, cs[e]);
      }
    }
  };


  // ---- prologue: slices 0..NSLOT-1 of the first tile
  int vb = bid;
  Rs ra, rb;
  tile_rs(vb, ra, rb);
#define VCX_PS_STAGE_U(U_)                                                                                   \
  stage_group(ra, rb, (U_), (U_), P0{}), stage_group(ra, rb, (U_), (U_), P1{}),                              \
      stage_group(ra, rb, (U_), (U_), P2{}), stage_group(ra, rb, (U_), (U_), P3{});
  VCX_PS_STAGE_U(0)
  VCX_PS_STAGE_U(1)
  VCX_PS_STAGE_U(2)
  VCX_PS_STAGE_U(3)
#undef VCX_PS_STAGE_U
  wait_vm<0>();  // the first NSLOT slices landed
  barrier();
  Frags f0, f1;
  load_x(0, 0), load_x(0, 2), load_x(0, 4), load_y(f0, 0), load_w(f0, 0, 0), load_w(f0, 0, 2);

  using VM = std::integral_constant<int, Gm::VMW>;
  using Tt = std::true_type;
  using Ff = std::false_type;
  while (true) {
    int m0, n0;
    coords(vb, m0, n0);
    const int vn = vb + G;
    const bool more = vn < tiles;
    Rs na, nb;  // the next tile's resources (the last tile re-stages its own first slices: never read)
    tile_rs(more ? vn : vb, na, nb);
    int s = 0;
    for (; s + 4 < nk; s += 2) {  // staging this tile's slices s + 4, s + 5
      step(s, f0, f1, ra, rb, s + 4, s < 3, Tt{}, VM{}, Tt{});
      step(s + 1, f1, f0, ra, rb, s + 5, s + 1 < 3, Tt{}, VM{}, Tt{});
    }
    // last 4 steps: the next tile's slices 0..3 go into the same ring
    step(s, f0, f1, na, nb, 0, false, Tt{}, VM{}, Tt{});
    step(s + 1, f1, f0, na, nb, 1, false, Tt{}, VM{}, Tt{});
    step(s + 2, f0, f1, na, nb, 2, false, Tt{}, VM{}, Tt{});
    if constexpr (reads_c2<EPI>()) {
      load_pre(m0, n0);  // lands behind the last step's MFMAs; its fragments are not read there
      // the 16 pre loads are younger loads than the awaited slice (loads retire in order)
      step(s + 3, f1, f0, na, nb, 3, false, Ff{}, std::integral_constant<int, 24>{}, Tt{});
      epilogue(m0, n0, Tt{});
      // the next tile's slice 0 (slot 0) landed before the epilogue's vmcnt(0)
      load_x(0, 0), load_x(0, 2), load_x(0, 4), load_y(f0, 0), load_w(f0, 0, 0), load_w(f0, 0, 2);
    } else {
      step(s + 3, f1, f0, na, nb, 3, false, Tt{}, VM{}, Tt{});
      epilogue(m0, n0, Tt{});  // the fragments of the next tile's slice 0 are in (x, f0) already
    }
    if (!more) break;
    vb = vn;
    ra = na;
    rb = nb;
  }
  // no final drain: the last epilogue's vmcnt(0) retired every LDS-DMA (the last tile re-stages
  // its own first slices as dummies), so only its stores are in flight, and those may outlive the
  // waves
}

}  // namespace gemm_ps
}  // namespace vcx

using namespace vcx;

bool vcx_gemm_ps_supported(int M, int N, int K, int epi) {
  using namespace gemm_ps;
  const bool known = epi == EPI_STORE || epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_DGELU ||
                     epi == EPI_BIAS_GELU_D || epi == EPI_DMUL;
  const bool bias = epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_GELU_D;
  return M > 0 && N > 0 && M % BM == 0 && N % BN == 0 && K % 128 == 0 && K >= 256 && known && (!bias || N <= BIAS_MAX);
}

int vcx_gemm_ps_grid(int M, int N, int grid_cap) {
  static const int ncu = [] {
    int dev = 0, n = 256;
    (void)hipGetDevice(&dev);
    (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
    return n;
  }();
  const int tiles = (M / gemm_ps::BM) * (N / gemm_ps::BN);
  int grid = grid_cap > 0 ? grid_cap : ncu;
  grid = grid < tiles ? grid & ~7 : tiles;  // a multiple of 8 (XCD remap) or one tile each
  return grid <= 0 ? tiles : grid;
}

void vcx_gemm_ps(const void* A, const void* B, void* C, void* C2, const void* bias, float* colsum, int M, int N,
                 int K, int lda, int ldb, int ldc, int epi, int grid_cap, hipStream_t s) {
  using namespace gemm_ps;
  static const bool attrs = [] {
    for (const void* k : {(const void*)gemm_ps_kernel<EPI_STORE>, (const void*)gemm_ps_kernel<EPI_BIAS>,
                          (const void*)gemm_ps_kernel<EPI_BIAS_GELU>, (const void*)gemm_ps_kernel<EPI_DGELU>,
                          (const void*)gemm_ps_kernel<EPI_BIAS_GELU_D>, (const void*)gemm_ps_kernel<EPI_DMUL>})
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, RING + 2 * BIAS_MAX);
    return true;
  }();
  (void)attrs;
  const int tilesN = N / BN, tiles = (M / BM) * tilesN;
  const int grid = vcx_gemm_ps_grid(M, N, grid_cap);
  const int lds =
      Geo::RINGB + (epi == EPI_BIAS || epi == EPI_BIAS_GELU || epi == EPI_BIAS_GELU_D ? (N * 2 + 15) & ~15 : 0);
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(grid), dim3(512), lds, s, (const bf16*)A, (const bf16*)B, (bf16*)C, (bf16*)C2,
                       (const bf16*)bias, colsum, M, N, K, lda, ldb, ldc, tilesN, tiles);
  };
  switch (epi) {
    case EPI_STORE: go(gemm_ps_kernel<EPI_STORE>); break;
    case EPI_BIAS: go(gemm_ps_kernel<EPI_BIAS>); break;
    case EPI_BIAS_GELU: go(gemm_ps_kernel<EPI_BIAS_GELU>); break;
    case EPI_BIAS_GELU_D: go(gemm_ps_kernel<EPI_BIAS_GELU_D>); break;
    case EPI_DMUL: go(gemm_ps_kernel<EPI_DMUL>); break;
    default: go(gemm_ps_kernel<EPI_DGELU>); break;
  }
}
