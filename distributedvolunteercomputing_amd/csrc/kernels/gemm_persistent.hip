// Persistent, role-split bf16 MFMA GEMM for gfx950 (MI355X) with fused epilogues.
//
//   C[M, N] = A[M, K] . op(B)      op(B) = B[N, K]^T   ("NT": x @ W^T, the forward GEMMs)
//                                  op(B) = B[K, N]     ("NN": dY @ W, the input gradients; no W^T copy)
//
// Why a second GEMM next to gemm.hip's tiled gemm_nt: at the GPT-2 shapes (K = 768: 24 K-slices
// per 256 x 256 tile, 3..12 rounds of tiles over the 256 CUs) the tiled kernel paid every round a
// cold prologue (the first slices from HBM) and a lockstep output burst (all 256 workgroups
// write their 128 KB tile at once), profiles/r2_gemm_nt.txt. Here:
//
//   * one 512-thread workgroup per CU walks its tiles (XCD-grouped order, tiles wl, wl + G, ...)
//     with ONE continuous LDS-DMA ring: the slices of tile t + 1 stream in while tile t finishes,
//     so a tile boundary costs no HBM latency;
//   * ROLE SPLIT. On CDNA4 vmcnt counts stores and loads together, in issue order: a wave that
//     stored its output tile could not wait for its next operand DMA without also waiting for
//     those stores (a 32 MB burst when every CU does it at once). So waves 4..7 ("loaders") issue
//     every operand DMA of the workgroup and never store, and waves 0..3 ("storers") issue every
//     output store and never DMA. All 8 waves run the MFMAs of their 128 x 64 sub-tile; at a tile
//     boundary every wave drops its accumulators (bias / GELU applied) into the ring slot that
//     is free at that moment (its fragments are already in registers), and the storers write the
//     tile out in full 128-B row segments (16 B per lane) and move on without waiting: the stores
//     drain under the next tile's MFMAs, and the loaders' counted waits only ever count DMA.
//   * main loop as gemm.hip: 256 x 256 tile, 8 waves as 2 (M) x 4 (N), v_mfma_f32_16x16x32_bf16,
//     4-slot ring of 32-deep K-slices (32 KB each), counted s_waitcnt vmcnt + raw s_barrier (two
//     slices stay in flight across each barrier), fragment reads double-buffered in registers,
//     XOR-swizzled LDS images (swizzle applied to the per-lane GLOBAL source address, guide rule
//     21), ds_read_b64_tr_b16 transposed reads for the N-major operand of the NN form (T10).
//   * a storer wave and a loader wave share each SIMD (waves w and w + 4), so the loader's DMA
//     issue slots sit beside the storer's MFMAs and vice versa.
//
// Epilogues: 0 store, 1 + bias, 2 pre = acc + bias -> C and gelu_tanh(pre) -> C2 (GPT-2 fc),
// 3 C = acc * gelu_tanh'(C2) and column sums of C added into colsum (GPT-2 fc2 input gradient +
// the fc bias gradient).
// Shapes: M % 256 == 0, K % 64 == 0, K >= 192 (the staging cursor may cross at most one tile
// boundary per tile); NT: N % 128 == 0 (a half tile at the right edge,
// e.g. the GPT-2 LM head, N = 50304); NN: N % 256 == 0.
// Reference analog: the per-frame compute hot loop /root/reference/worker.py:249 (OpenCV DNN),
// whose cost is 87 % pointwise GEMM; the training GEMMs are BASELINE's north star.
#include <type_traits>

#include "vcx_common.h"

namespace vcx {
namespace gemmp {

typedef short sx8 __attribute__((ext_vector_type(8)));
typedef short sx4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BN = 256, BKS = 32, NT = 512, NSLOT = 4;
constexpr int ROWB = BKS * 2;                 // 64 B: one row of a K-major slice image
constexpr int TROW = BN * 2;                  // 512 B: one k-row of an N-major slice image
constexpr int HALF = BM * ROWB;               // 16 KB: one operand of a slice (either layout)
constexpr int SLOT = 2 * HALF;                // 32 KB
constexpr int RING = NSLOT * SLOT;            // 128 KB
constexpr int AUX_BIAS = RING;                // 256 bf16 of bias for the tile
constexpr int AUX_CS = RING + 512;            // 2 x 256 fp32 column-sum partials
constexpr int LDS_BYTES = RING + 512 + 2048;  // 133632 (multiple of 16)
constexpr int STG = 4096;                     // epilogue staging per wave: 32 rows x 128 B

enum Epi { EPI_STORE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_DGELU = 3 };

// K-major image: 64-B rows, 16-B chunk swizzle F[(row >> 2) & 3] = {0, 2, 3, 1}
__device__ __forceinline__ int swz(int row) { return (0x78 >> (((row >> 2) & 3) * 2)) & 3; }
// N-major image: 512-B k-rows, chunk swizzle 2 * ((r & 3) | (r >> 3 & 1) << 2)
__device__ __forceinline__ int tn_swz(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }

// s_waitcnt vmcnt(N) lgkmcnt(0) (N < 64; vmcnt bits [3:0] and [15:14], expcnt left at its maximum)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 64, "vmcnt field");
  __builtin_amdgcn_s_waitcnt(0x0070 | (N & 15) | ((N >> 4) << 14));
}
__device__ __forceinline__ void wait_lgkm() { __builtin_amdgcn_s_waitcnt(0xC07F); }
// raw barrier the compiler may not move LDS accesses across (the builtin is IntrNoMem)
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

__device__ __forceinline__ void glds16(const bf16* g, char* lds) {
  __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)g,
                                   (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ sx8 tr_frag(const char* p0, const char* p1) {
  const sx4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sx4*)(p0));
  const sx4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sx4*)(p1));
  return sx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

__device__ __forceinline__ float gelu_tanh(float x) {
  // 0.5 x (1 + tanh(u)) = x * sigmoid(2u), u = sqrt(2/pi) (x + 0.044715 x^3)
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x * x, x);
  return x / (1.f + __expf(-u2));
}

__device__ __forceinline__ float gelu_tanh_grad(float x) {
  const float x2 = x * x;
  const float u2 = 1.5957691216057308f * fmaf(0.044715f * x, x2, x);
  const float s = 1.f / (1.f + __expf(-u2));
  return fmaf(x * s * (1.f - s), 1.5957691216057308f * fmaf(0.134145f, x2, 1.f), s);
}


template <int EPI, bool BT>
__global__ void __launch_bounds__(NT, 1)
    gemm_p_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, bf16* __restrict__ C,
                  bf16* __restrict__ C2, const bf16* __restrict__ bias, float* __restrict__ colsum, int M, int N,
                  int K, int lda, int ldb, int ldc, int tilesM, int tilesN) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3, v = wid & 3;

  // ---- persistent tile walk: XCD-aware bijective remap of the workgroup index (workgroups that
  // share an XCD get consecutive indices), then tiles wl, wl + G, ... in GROUP_M-row-panel blocks
  const int G = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = G >> 3, r8 = G & 7;
  const int wl = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int tiles = tilesM * tilesN;
  const int my_tiles = (tiles - wl + G - 1) / G;  // >= 1: G <= tiles
  const int nk = K / BKS;                          // even, >= 6
  constexpr int GROUP_M = 4;
  auto coords = [&](int t, int& m0, int& n0) {  // t past the end: the last tile (dummy staging)
    const int L = wl + min(t, my_tiles - 1) * G;
    const int per_group = GROUP_M * tilesN;
    const int gfirst = (L / per_group) * GROUP_M;
    const int gsize = min(tilesM - gfirst, GROUP_M);
    const int rr = L - (L / per_group) * per_group;
    m0 = (gfirst + rr % gsize) * BM;
    n0 = (rr / gsize) * BN;
  };

  // ---- fragment reads (every wave): lane l -> row (l & 15) of a 16-row block, k chunk (l >> 4)
  const int frow = lane & 15;
  const int foff = frow * ROWB + (((lane >> 4) ^ swz(frow)) << 4);
  const int xa_off = (wm * 128) * ROWB + foff;
  const int wb_off = HALF + (wn * 64) * ROWB + foff;
  // NN: transposed reads of the N-major B image (lane group g = l >> 4 takes k-rows 8g + 4h + q)
  const int tg = lane >> 4, te = lane & 15, tq = te >> 2, tp = te & 3;
  const int tr0 = 8 * tg + tq, tr1 = tr0 + 4;
  const int tf0 = tn_swz(tr0), tf1 = tn_swz(tr1);
  const int thalf8 = (tp & 1) * 8, thchunk = tp >> 1;
  auto toff = [&](int c, int rr, int ff) { return rr * TROW + ((((c >> 3) ^ ff) + thchunk) << 4) + thalf8; };

  // A fragments x[i] (row block i of the wave's 128 rows) and B fragments w[j] (column block j)
  // x[0..5] are single-buffered (refilled right behind the MFMA group that used them); the last
  // group's rows (6, 7) and the B fragments alternate between two named sets, so every read of
  // the next slice is issued before the step's last MFMA group
  sx8 x[6], yA[2], yB[2], wA[4], wB[4];
  auto load_x = [&](int so, auto I) {
    constexpr int i = decltype(I)::value;
    x[i] = *(const sx8*)(smem + so + xa_off + i * 16 * ROWB);
    x[i + 1] = *(const sx8*)(smem + so + xa_off + (i + 1) * 16 * ROWB);
  };
  auto load_y = [&](sx8 (&y)[2], int so) {
    y[0] = *(const sx8*)(smem + so + xa_off + 6 * 16 * ROWB);
    y[1] = *(const sx8*)(smem + so + xa_off + 7 * 16 * ROWB);
  };
  auto load_w = [&](sx8 (&w)[4], int so) {
    if constexpr (!BT) {
#pragma unroll
      for (int j = 0; j < 4; ++j) w[j] = *(const sx8*)(smem + so + wb_off + j * 16 * ROWB);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int c = wn * 64 + 16 * j;
        w[j] = tr_frag(smem + so + HALF + toff(c, tr0, tf0), smem + so + HALF + toff(c, tr1, tf1));
      }
    }
  };

  f32x4 acc[8][4];
  auto mma = [&](const sx8 (&y)[2], const sx8 (&w)[4], auto I0, auto ZC) {  // row blocks I0, I0 + 1
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = decltype(I0)::value; i < decltype(I0)::value + 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const sx8& xf = i < 6 ? x[i < 6 ? i : 0] : y[i - 6 >= 0 ? i - 6 : 0];
        if constexpr (decltype(ZC)::value)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xf, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        else
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(w[j], xf, acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  using I0c = std::integral_constant<int, 0>;
  using I2c = std::integral_constant<int, 2>;
  using I4c = std::integral_constant<int, 4>;
  using I6c = std::integral_constant<int, 6>;
  using Tt = std::true_type;
  using Ff = std::false_type;

  auto run = [&](auto LD) {
    constexpr bool LOADER = decltype(LD)::value;

    // ---- loader-side staging cursor: slice st_k of tile st_t; the pieces of a slice are 16 A
    // pieces (16 rows x 64 B) and 16 B pieces (NT: 16 rows x 64 B; NN: 2 k-rows x 512 B); loader
    // wave v moves pieces v, v + 4, v + 8, v + 12 of each. Per-lane offsets are tile-invariant.
    const int prow = lane >> 2;
    const int a_off = (v * 16 + prow) * lda + ((lane & 3) ^ swz(prow)) * 8;
    int b_off0, b_off1;
    if constexpr (!BT) {
      b_off0 = (v * 16 + prow) * ldb + ((lane & 3) ^ swz(prow)) * 8;
      b_off1 = b_off0;
    } else {
      const int srow = 2 * v + (lane >> 5);  // piece v + 4j: k-rows srow + 8j
      b_off0 = srow * ldb + (((lane & 31) ^ tn_swz(srow)) * 8);
      b_off1 = srow * ldb + (((lane & 31) ^ tn_swz(srow + 8)) * 8);
    }
    const bf16 *sa = A, *sb = B, *nsa = A, *nsb = B;
    int bhalf = 0, nbhalf = 0;  // NT: rows of B pieces j = 2, 3 (128, or 0 past the right edge)
    int st_k = 0;
    auto bases = [&](int t, const bf16*& pa, const bf16*& pb, int& bh) {
      int m0, n0;
      coords(t, m0, n0);
      pa = A + (int64_t)m0 * lda;
      if constexpr (!BT) {
        pb = B + (int64_t)n0 * ldb;
        bh = (n0 + 128 < N) ? 128 : 0;
      } else {
        pb = B + n0;
        bh = 0;
      }
    };
    auto stage_piece = [&](char* slotp, auto P) {  // P: 0..3 A pieces, 4..7 B pieces (compile time)
      constexpr int p = decltype(P)::value, j = p & 3;
      char* dst = slotp + (p < 4 ? 0 : HALF) + (v + 4 * j) * 1024;
      if constexpr (p < 4) {
        glds16(sa + (int64_t)(64 * j) * lda + st_k * BKS + a_off, dst);
      } else if constexpr (!BT) {
        const int ro = j < 2 ? 64 * j : bhalf + 64 * (j - 2);
        glds16(sb + (int64_t)ro * ldb + st_k * BKS + b_off0, dst);
      } else {
        glds16(sb + (int64_t)(st_k * BKS + 8 * j) * ldb + ((j & 1) ? b_off1 : b_off0), dst);
      }
    };
    auto advance = [&]() {  // branch-free: the next tile's bases are precomputed
      ++st_k;
      const bool wrap = st_k == nk;
      st_k = wrap ? 0 : st_k;
      sa = wrap ? nsa : sa;
      sb = wrap ? nsb : sb;
      bhalf = wrap ? nbhalf : bhalf;
    };
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    using P2 = std::integral_constant<int, 2>;
    using P3 = std::integral_constant<int, 3>;
    using P4 = std::integral_constant<int, 4>;
    using P5 = std::integral_constant<int, 5>;
    using P6 = std::integral_constant<int, 6>;
    using P7 = std::integral_constant<int, 7>;
    auto stage_all = [&](char* slotp) {
      stage_piece(slotp, P0{}), stage_piece(slotp, P1{}), stage_piece(slotp, P2{}), stage_piece(slotp, P3{});
      stage_piece(slotp, P4{}), stage_piece(slotp, P5{}), stage_piece(slotp, P6{}), stage_piece(slotp, P7{});
    };

    // ---- one K-step: slice s is in registers (x, wc). Loaders: retire their DMA of slice s + 1
    // (the two later slices stay in flight: 16 ops); everyone: barrier (slice s + 1 visible, the
    // slot of slice s no longer read). Loaders issue slice s + 4 into that slot, 2 pieces per MFMA
    // group. Each MFMA group (2 row blocks) frees its two A fragments, which are refilled from
    // slice s + 1 right behind it; the B fragments of slice s + 1 go to the other set (wn).
    auto step = [&](int s, sx8(&yc)[2], sx8(&wc)[4], sx8(&yn)[2], sx8(&wnx)[4], auto ZC, auto VW) {
      if constexpr (LOADER && decltype(VW)::value) wait_vm<16>();
      else wait_lgkm();
      barrier();
      char* slotp = smem + (s & 3) * SLOT;
      const int so = ((s + 1) & 3) * SLOT;
      if constexpr (LOADER) stage_piece(slotp, P0{}), stage_piece(slotp, P4{});
      __builtin_amdgcn_sched_barrier(0);
      mma(yc, wc, I0c{}, ZC);
      __builtin_amdgcn_sched_barrier(0);
      load_x(so, I0c{});
      load_w(wnx, so);
      if constexpr (LOADER) stage_piece(slotp, P1{}), stage_piece(slotp, P5{});
      __builtin_amdgcn_sched_barrier(0);
      mma(yc, wc, I2c{}, ZC);
      __builtin_amdgcn_sched_barrier(0);
      load_x(so, I2c{});
      load_y(yn, so);
      if constexpr (LOADER) stage_piece(slotp, P2{}), stage_piece(slotp, P6{});
      __builtin_amdgcn_sched_barrier(0);
      mma(yc, wc, I4c{}, ZC);
      __builtin_amdgcn_sched_barrier(0);
      load_x(so, I4c{});
      if constexpr (LOADER) {
        stage_piece(slotp, P3{}), stage_piece(slotp, P7{});
        advance();
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(yc, wc, I6c{}, ZC);
    };

    // ---- epilogue of tile (m0, n0); s = the first slice of the next tile, whose fragments are in
    // registers already, so the ring slot X = s & 3 is free until the next step's barrier
    auto epilogue = [&](int m0, int n0, int s) {
      if constexpr (LOADER) wait_vm<16>();  // slice s + 1 landed (the next step waits for nothing)
      else wait_lgkm();
      // lane-derived offsets are recomputed per epilogue (opaque lane id): hoisted above the tile
      // loop they would stay live through the main loop and spill
      int ln = lane;
      asm volatile("" : "+v"(ln));
      const int fr = ln & 15, cl = 4 * (ln >> 4);
      bf16* const lbias = (bf16*)(smem + AUX_BIAS);
      if constexpr (!LOADER && (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU)) {
        lbias[wid * 64 + ln] = bias[min(n0 + wid * 64 + ln, N - 1)];
      }
      barrier();  // slot X no longer read by anyone; bias visible
      char* const xslot = smem + (s & 3) * SLOT;
      char* const stg = xslot + wid * STG;
      // a wave's staged 32 x 64 block: 128-B rows, 16-B chunks XOR-swizzled by (row & 7)
      auto sidx = [&](int r, int c) { return r * 128 + (((c >> 3) ^ (r & 7)) << 4) + ((c >> 2) & 1) * 8; };
      // storers: 16 B per lane, lane -> chunk k8 of row rl of an 8-row x 128-B piece; buffer stores
      // on the tile's first row with a 32-bit per-lane offset and the row offset in an SGPR
      const int k8 = ln & 7, rl = ln >> 3;
      const int colg = n0 + wn * 64 + k8 * 8;  // global column of this lane's 8 outputs
      const bool colok = colg < N;
      const int voff = (rl * ldc + colg) * 2;
      const int lsrc = rl * 128 + ((k8 ^ rl) << 4);  // + region + 1024 * it
      const int64_t tbytes = (int64_t)(M - m0) * ldc * 2;
      const int nrec = tbytes < 0x7FFFFFF0 ? (int)tbytes : 0x7FFFFFF0;
      typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
      auto rsrc = [&](const bf16* base) {
        return __builtin_amdgcn_make_buffer_rsrc((void*)(base + (int64_t)m0 * ldc), (short)0, nrec, 0x00020000);
      };
      auto st16 = [&](const decltype(rsrc(C))& rs, int row, const bf16x8& val) {  // row inside the tile
        if (colok) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, val), rs, voff, row * ldc * 2, 0);
      };
      auto flush = [&](int rb) {  // the staged 32-row blocks of waves (v, v + 4) -> tile rows rb + ...
        if constexpr (!LOADER) {
          const auto rs = rsrc(C);
#pragma unroll
          for (int h = 0; h < 2; ++h)
#pragma unroll
            for (int it = 0; it < 4; ++it) {
              const bf16x8 val = *(const bf16x8*)(xslot + (v + 4 * h) * STG + lsrc + 1024 * it);
              st16(rs, 128 * h + rb + 8 * it, val);
            }
        }
      };
      if constexpr (EPI == EPI_STORE || EPI == EPI_BIAS) {
#pragma unroll
        for (int rnd = 0; rnd < 4; ++rnd) {
          if (rnd) barrier();  // the storers are done reading the previous round
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float bj[4] = {0.f, 0.f, 0.f, 0.f};
            if constexpr (EPI == EPI_BIAS) {
              const bf16x4 bv = *(const bf16x4*)(lbias + wn * 64 + 16 * j + cl);
#pragma unroll
              for (int t = 0; t < 4; ++t) bj[t] = (float)bv[t];
            }
#pragma unroll
            for (int ii = 0; ii < 2; ++ii) {
              bf16x4 o;
#pragma unroll
              for (int t = 0; t < 4; ++t) o[t] = (bf16)(acc[2 * rnd + ii][j][t] + bj[t]);
              *(bf16x4*)(stg + sidx(16 * ii + fr, 16 * j + cl)) = o;
            }
          }
          wait_lgkm();
          barrier();
          flush(32 * rnd);
          wait_lgkm();
        }
      } else if constexpr (EPI == EPI_BIAS_GELU) {
        // 16-row rounds: pre in rows 0..15 of the staging block, gelu(pre) in rows 16..31
#pragma unroll
        for (int rnd = 0; rnd < 8; ++rnd) {
          if (rnd) barrier();
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const bf16x4 bv = *(const bf16x4*)(lbias + wn * 64 + 16 * j + cl);
            bf16x4 o, g;
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              o[t] = (bf16)(acc[rnd][j][t] + (float)bv[t]);
              g[t] = (bf16)gelu_tanh((float)o[t]);
            }
            *(bf16x4*)(stg + sidx(fr, 16 * j + cl)) = o;
            *(bf16x4*)(stg + sidx(16 + fr, 16 * j + cl)) = g;
          }
          wait_lgkm();
          barrier();
          if constexpr (!LOADER) {
            const auto rc = rsrc(C), rg = rsrc(C2);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int it = 0; it < 4; ++it) {  // it 0, 1: pre rows; 2, 3: gelu rows
                const bf16x8 val = *(const bf16x8*)(xslot + (v + 4 * h) * STG + lsrc + 1024 * it);
                st16(it < 2 ? rc : rg, 128 * h + 16 * rnd + 8 * (it & 1), val);
              }
          }
          wait_lgkm();
        }
      } else {  // EPI_DGELU: C = acc * gelu'(pre = C2), column sums of C into colsum
        float cs[4][4];
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) cs[j][t] = 0.f;
        bf16x8 pre[2][4];
        auto load_pre = [&](int rnd) {  // storers: this round's pre rows of waves (v, v + 4)
          if constexpr (!LOADER) {
            const auto rp = rsrc(C2);
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int it = 0; it < 4; ++it)
                pre[h][it] = __builtin_bit_cast(
                    bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rp, voff, (128 * h + 32 * rnd + 8 * it) * ldc * 2, 0));
          }
        };
        load_pre(0);
#pragma unroll
        for (int rnd = 0; rnd < 4; ++rnd) {
          if (rnd) barrier();
          if constexpr (!LOADER) {  // pre rows -> both staging blocks (same swizzled image)
#pragma unroll
            for (int h = 0; h < 2; ++h)
#pragma unroll
              for (int it = 0; it < 4; ++it) *(bf16x8*)(xslot + (v + 4 * h) * STG + lsrc + 1024 * it) = pre[h][it];
            if (rnd < 3) load_pre(rnd + 1);  // in flight beside this round's work and stores
          }
          wait_lgkm();
          barrier();
#pragma unroll
          for (int ii = 0; ii < 2; ++ii)
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              char* p = stg + sidx(16 * ii + fr, 16 * j + cl);
              const bf16x4 pv = *(const bf16x4*)p;
              bf16x4 o;
#pragma unroll
              for (int t = 0; t < 4; ++t) {
                o[t] = (bf16)(acc[2 * rnd + ii][j][t] * gelu_tanh_grad((float)pv[t]));
                cs[j][t] += (float)o[t];
              }
              *(bf16x4*)p = o;
            }
          wait_lgkm();
          barrier();
          flush(32 * rnd);
          wait_lgkm();
        }
        // column sums: 16 lanes share a column set; waves (v, v + 4) share columns
        float* const lcs = (float*)(smem + AUX_CS);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int t = 0; t < 4; ++t) {
            float x = cs[j][t];
            x += __shfl_xor(x, 1, 64);
            x += __shfl_xor(x, 2, 64);
            x += __shfl_xor(x, 4, 64);
            x += __shfl_xor(x, 8, 64);
            if (fr == 0) lcs[wm * 256 + wn * 64 + 16 * j + cl + t] = x;
          }
        wait_lgkm();
        barrier();
        if constexpr (!LOADER) {
          const int c = n0 + wn * 64 + ln;
          const float x = lcs[wn * 64 + ln] + lcs[256 + wn * 64 + ln];
          if (c < N) atomicAdd(colsum + c, x);
        }
      }
    };

    // ---- prologue: slices 0..3 in flight, slice 0 in registers, slice 1 landed
    if constexpr (LOADER) {
      bases(0, sa, sb, bhalf);
      bases(1, nsa, nsb, nbhalf);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        stage_all(smem + i * SLOT);
        advance();
      }
      wait_vm<24>();
    }
    barrier();
    load_x(0, I0c{});
    load_x(0, I2c{});
    load_x(0, I4c{});
    load_y(yA, 0);
    load_w(wA, 0);
    if constexpr (LOADER) wait_vm<16>();
    else wait_lgkm();

    int s = 0;
    for (int t = 0; t < my_tiles; ++t) {
      if constexpr (LOADER) {
        if (t > 0) bases(t + 1, nsa, nsb, nbhalf);  // the cursor enters tile t + 1 during tile t
      }
      step(s, yA, wA, yB, wB, Tt{}, Ff{});  // accumulators start at zero; slice s + 1 landed already
      step(s + 1, yB, wB, yA, wA, Ff{}, Tt{});
      s += 2;
      for (int kk = 2; kk < nk; kk += 2, s += 2) {
        step(s, yA, wA, yB, wB, Ff{}, Tt{});
        step(s + 1, yB, wB, yA, wA, Ff{}, Tt{});
      }
      int m0, n0;
      coords(t, m0, n0);
      epilogue(m0, n0, s);
    }
    if constexpr (LOADER) wait_vm<0>();  // no LDS-DMA may be in flight when the wave ends
  };

  if (wid >= 4) run(Tt{});
  else run(Ff{});
}

}  // namespace gemmp
}  // namespace vcx

using namespace vcx;

// layout: 0 = NT (B [N, K]), 1 = NN (B [K, N])
bool vcx_gemm_p_supported(int M, int N, int K, int layout) {
  if (M <= 0 || N <= 0 || K < 192 || M % gemmp::BM || K % 64) return false;
  return layout == 0 ? N % 128 == 0 : N % 256 == 0;
}

static int vcx_num_cus() {
  static int n = [] {
    int dev = 0, c = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || c <= 0) c = kNumCU;
    return c;
  }();
  return n;
}

// C = A . op(B) with epilogue `epi`; colsum (epi 3) must be zeroed by the caller.
void vcx_gemm_p(const void* A, const void* B, void* C, void* C2, const void* bias, float* colsum, int M, int N, int K,
                int lda, int ldb, int ldc, int epi, int layout, hipStream_t s) {
  using namespace gemmp;
  const int tilesM = M / BM, tilesN = (N + BN - 1) / BN, tiles = tilesM * tilesN;
  const int G = tiles < vcx_num_cus() ? tiles : vcx_num_cus();
  static const bool attrs = [] {
    for (const void* k :
         {(const void*)gemm_p_kernel<EPI_STORE, false>, (const void*)gemm_p_kernel<EPI_BIAS, false>,
          (const void*)gemm_p_kernel<EPI_BIAS_GELU, false>, (const void*)gemm_p_kernel<EPI_DGELU, false>,
          (const void*)gemm_p_kernel<EPI_STORE, true>, (const void*)gemm_p_kernel<EPI_BIAS, true>,
          (const void*)gemm_p_kernel<EPI_BIAS_GELU, true>, (const void*)gemm_p_kernel<EPI_DGELU, true>})
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    return true;
  }();
  (void)attrs;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(G), dim3(NT), LDS_BYTES, s, (const bf16*)A, (const bf16*)B, (bf16*)C, (bf16*)C2,
                       (const bf16*)bias, colsum, M, N, K, lda, ldb, ldc, tilesM, tilesN);
  };
  if (layout == 0) {
    switch (epi) {
      case EPI_STORE: go(gemm_p_kernel<EPI_STORE, false>); break;
      case EPI_BIAS: go(gemm_p_kernel<EPI_BIAS, false>); break;
      case EPI_BIAS_GELU: go(gemm_p_kernel<EPI_BIAS_GELU, false>); break;
      default: go(gemm_p_kernel<EPI_DGELU, false>); break;
    }
  } else {
    switch (epi) {
      case EPI_STORE: go(gemm_p_kernel<EPI_STORE, true>); break;
      case EPI_BIAS: go(gemm_p_kernel<EPI_BIAS, true>); break;
      case EPI_BIAS_GELU: go(gemm_p_kernel<EPI_BIAS_GELU, true>); break;
      default: go(gemm_p_kernel<EPI_DGELU, true>); break;
    }
  }
}
