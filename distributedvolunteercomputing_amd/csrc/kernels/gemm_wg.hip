// Weight-gradient GEMM for gfx950 (the default weight gradient of ops/linear.py):
//
//   Cpart[s][M, N] = sum over tokens k of split s of A[k, M]^T . B[k, N]      (fp32 partials)
//   out (bf16 [M, N]) (+)= sum_s Cpart[s]                                    (splitk_sum_kernel)
//
// The weight gradient of a token-major linear layer, dW[out, in] = dY[tok, out]^T X[tok, in]: both
// operands are TOKEN-major (the reduction runs over their row index), the output is small (9..36 tiles
// of 256 x 256 at GPT-2-small), so the token axis is split over the CUs and every split streams its
// token range of both operands once. Structure:
//   * 256 x 256 tile per 512-thread workgroup (8 waves as 2 (M) x 4 (N), 128 x 64 each,
//     v_mfma_f32_16x16x32_bf16), 4-slot LDS ring of 32-token slices staged by LDS-DMA, counted vmcnt +
//     raw s_barrier (two slices in flight across every barrier), fragments read TRANSPOSED out of the
//     token-row LDS image by ds_read_b64_tr_b16 (cdna guide T10); A rows 0..5 single-buffered, rows 6, 7
//     and the B fragments double-buffered in registers.
//   * the LDS-DMA is issued by inline asm (dma16), not by the buffer/global_load_lds builtins. With the
//     builtins, hipcc (ROCm 7.2) cannot tell a pending LDS-DMA from the slot a later
//     ds_read_b64_tr_b16 reads and drains vmcnt(0) in front of the transposed fragment reads -- 8 full
//     drains per step in the earlier gemm_tn, whose "waves parked on vmcnt 73 % of the time"
//     (profiles/r2_gemm_tn.txt) were those drains, not memory latency. Invisible to that pass, the
//     DMA is ordered only by this kernel's own counted waits: 1165-1229 TF/s at the GPT-2 shapes
//     against the library's 808-978 (profiles/r5_gemm_wg.txt).
//   * measured and dropped (profiles/r5_gemm_wg.txt): wave-role loads (waves 0-3 staging, 4-7 touching
//     slice t + PF into L2 without ever waiting, the tiles of a split sharing the touches) -- once the
//     drains were gone the prefetch only cost (pf 4..12: 0-7 % slower than none).
//   * XCD-aware order over (split, tile): the tiles of one split (same token rows) run side by side
//     on one XCD and share its L2.
// Reference analog: none (the reference trains nothing; SURVEY.md §2.9 north-star trainer).
#include <type_traits>

#include <algorithm>
#include <cstdlib>

#include "vcx_common.h"

namespace vcx {
namespace gemm_wg {

typedef short sx8 __attribute__((ext_vector_type(8)));
typedef short sx4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

constexpr int BM = 256, BN = 256, BKS = 32, NT = 512;
constexpr int TROW = 512;                      // bytes per token row of a 256-wide operand slice
constexpr int TSLOT_A = BKS * TROW;            // 16 KB
constexpr int SLOT_BYTES = 2 * TSLOT_A;        // 32 KB: A and B slices
constexpr int LDS_BYTES = 4 * SLOT_BYTES;      // 128 KB ring

// 16-B chunk swizzle of a token row: F(r) = 2 (r & 3 | (r >> 3 & 1) << 2); a half-wave's two transposed
// reads touch 8 rows (q = r & 3 and the group parity r >> 3 & 1) x 2 chunks, spread over all 16 bank
// slots (conflict-free). LDS-DMA writes lane-linearly, so the swizzle goes on the GLOBAL source address.
__device__ __forceinline__ int swz(int r) { return ((r & 3) | (((r >> 3) & 1) << 2)) << 1; }

__device__ __forceinline__ sx8 tr_frag(const char* p0, const char* p1) {
  const sx4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sx4*)(p0));
  const sx4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sx4*)(p1));
  return sx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// buffer resource words over [base, base + bytes) for inline asm ("s" operand): wave-uniform base and
// size (SGPRs), 32-bit per-lane offsets
__device__ __forceinline__ u32x4 desc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  return u32x4{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, (unsigned)bytes, 0x00020000u};
}

// One 1-KB LDS-DMA piece (16 B per lane to LDS base + 16 lane) as inline asm, M0 = the LDS byte address.
// Why not __builtin_amdgcn_raw_ptr_buffer_load_lds: hipcc (ROCm 7.2) cannot tell a pending LDS-DMA from
// the slot a later ds_read_b64_tr_b16 reads, so it drained vmcnt(0) in front of every transposed
// fragment read of the step -- 8 full drains per step in gemm_tn, the whole pipeline serialised (the
// "waves parked on vmcnt" of profiles/r2_gemm_tn.txt). Issued as asm, the DMA is invisible to that
// pass; the kernel's own counted waits (wait_vm) order it. `s_nop 0`: the M0 write -> LDS-DMA hazard.
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
__device__ __forceinline__ void wait_lgkm0() { __builtin_amdgcn_s_waitcnt(0xC07F); }  // vmcnt 63: no VM wait
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

struct Frags {
  sx8 y[2];  // A fragments of row blocks 6, 7
  sx8 w[4];  // B fragments: the wave's 4 column blocks of 16 (output columns)
};

// Implicit 3x3 convolution operand (IMPL): B is the NHWC input x [imgs, H, W, Cin] of a 3x3 convolution
// (pad 1, stride st) and the kernel's B matrix is its patch matrix P[token, (ky, kx, c)] -- token = output
// pixel (img, oy, ox), P = x[img, oy st + ky - 1, ox st + kx - 1, c] (0 outside the image) -- so
// out[Cout, 9 Cin] = dY^T P is the convolution's weight gradient in the channels-last weight layout
// [Cout][ky][kx][Cin], without an im2col matrix. Each lane's 8 columns lie in one tap (Cin % 8 == 0; a
// 256-column block of P spans 2 taps at Cin = 128); past the last tap (9 Cin % 256 != 0: the ragged last
// column block) the lane stages zeros and those output columns are not stored.
struct ConvG {
  int H, W, Ho, Wo, Cin, st, xbytes;
};

// NLW = the waves that stage the ring: 8 (every wave moves 4 of a slice's 32 pieces; the default) or 4
// (waves 0-3 move 8 each, waves 4-7 only compute: 1-3 % slower, profiles/r5_gemm_wg.txt; kept as the
// tested alternative geometry)
template <int NLW, bool IMPL>
__global__ void __launch_bounds__(NT, 1)
    gemm_wg_kernel(const bf16* __restrict__ A, const bf16* __restrict__ B, float* __restrict__ Cpart, int M, int N,
                   int K, int lda, int ldb, int tilesN, int tiles, int splits, ConvG cg) {
  static_assert(NLW == 4 || NLW == 8, "loader waves");
  static_assert(!IMPL || NLW == 8, "the implicit operand is staged by all 8 waves");
  constexpr int PPO = 16 / NLW;   // pieces of one operand per loader wave
  constexpr int OPS = 2 * PPO;    // LDS-DMA ops per slice per loader wave
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wid >> 2, wn = wid & 3;

  // ---- XCD-aware bijective order over (split, tile): consecutive logical ids share an XCD, so the
  // tiles of one split (same token range) run side by side there and share its L2
  const int nwg = gridDim.x, bid = blockIdx.x;
  const int xcd = bid & 7, q8 = nwg >> 3, r8 = nwg & 7;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + (bid >> 3);
  const int split = wg / tiles, tile = wg - split * tiles;
  const int tm = tile / tilesN, tn = tile - tm * tilesN;
  const int m0 = tm * BM, n0 = tn * BN;
  const int nb64 = K >> 6;
  const int kb0 = (int)((int64_t)split * nb64 / splits), kb1 = (int)((int64_t)(split + 1) * nb64 / splits);
  const int kbeg = kb0 * 64;
  const int nk = (kb1 - kb0) * 2;  // slices of 32 tokens: even, >= 6 (host: K / 192 >= splits)

  // ---- staging: piece P (0..15) of an operand slice = token rows 2P, 2P + 1 (64 lanes x 16 B); loader
  // wave w moves pieces w + NLW i (i < PPO) of A and of B. Lane l: row 2P + (l >> 5), physical chunk
  // l & 31, holding logical chunk (l & 31) ^ F(row). F depends on the row's bit 3: for NLW = 8 the rows
  // of a wave's pieces are 16 apart (one F), for NLW = 4 8 apart (F alternates with i & 1). Buffer
  // resources over this split's token rows of the tile's panels (host check: they fit 31 bits); the
  // slice and the 16-row steps go into soffset.
  const int ntok = (kb1 - kb0) * 64;
  const int lw = wid & (NLW - 1);
  const int row_e = 2 * lw + (lane >> 5), row_o = row_e + 8;
  const int ch_e = ((lane & 31) ^ swz(row_e)) * 8, ch_o = ((lane & 31) ^ swz(row_o)) * 8;
  const bf16* a_base = A + (int64_t)kbeg * lda + m0;
  const bf16* b_base = IMPL ? B : B + (int64_t)kbeg * ldb + n0;
  // (byte counts and slice offsets computed unsigned; the host keeps a split's panel under 2 GB)
  const u32x4 ra = desc(a_base, (unsigned)ntok * (unsigned)lda * 2u),
              rb = IMPL ? desc(B, (unsigned)cg.xbytes) : desc(b_base, (unsigned)ntok * (unsigned)ldb * 2u);
  // ragged last row panel (M % 256 = 128): the lanes of columns past M re-read the panel's last valid chunk
  // (their output rows are not stored), so no load leaves the operand -- the LM head's logit gradient ends
  // exactly at its allocation's end
  const int cha_e = min(ch_e, M - m0 - 8), cha_o = min(ch_o, M - m0 - 8);
  const int va_e = (row_e * lda + cha_e) * 2, va_o = (row_o * lda + cha_o) * 2;
  const int vb_e = (row_e * ldb + ch_e) * 2, vb_o = (row_o * ldb + ch_o) * 2;
  const unsigned a_sl = BKS * lda * 2, b_sl = BKS * ldb * 2;  // bytes per slice (32 rows)
  char* const lds_w = smem + lw * 1024;

  // IMPL: the output pixel of each of this lane's B rows (row_e + 16 i of the NEXT slice to stage), advanced
  // by 32 tokens after every op that stages it (the ops of one piece are issued in slice order); a row
  // whose tap falls outside the image gets an offset past the resource, which the buffer load returns as 0.
  // The lane's tap and channel come from its own patch column n0 + ch_e (the same in every row it stages)
  int timg[PPO], toy[PPO], tox[PPO], tdy = 0, tdx = 0, tc0 = 0;
  if constexpr (IMPL) {
    const int pcol = n0 + ch_e, tap = pcol / cg.Cin;
    tc0 = pcol - tap * cg.Cin;
    tdy = tap < 9 ? tap / 3 - 1 : (1 << 24);  // past the last tap: never inside the image
    tdx = tap - 3 * (tap / 3) - 1;
    const int hw = cg.Ho * cg.Wo;
#pragma unroll
    for (int i = 0; i < PPO; ++i) {
      const int t = kbeg + row_e + 16 * i, img = t / hw, rem = t - img * hw, oy = rem / cg.Wo;
      timg[i] = img;
      toy[i] = oy;
      tox[i] = rem - oy * cg.Wo;
    }
  }

  // op o (0..OPS-1) of slice s: A pieces for o < PPO (i = o), B pieces after (i = o - PPO)
  auto stage_op = [&](int s, int o) {
    char* slot = lds_w + (s & 3) * SLOT_BYTES;
    const int i = o % PPO;
    const bool odd = NLW == 4 && (i & 1);
    const int r16 = NLW == 4 ? (i >> 1) : i;  // 16-row steps
    if (o < PPO) {
      dma16(ra, odd ? va_o : va_e, (int)((unsigned)s * a_sl + (unsigned)r16 * (a_sl >> 1)), slot + i * NLW * 1024);
    } else if constexpr (IMPL) {
      const int iy = toy[i] * cg.st + tdy, ix = tox[i] * cg.st + tdx;
      const bool in = (unsigned)iy < (unsigned)cg.H && (unsigned)ix < (unsigned)cg.W;
      const int voff = in ? (((timg[i] * cg.H + iy) * cg.W + ix) * cg.Cin + tc0) * 2 : cg.xbytes;
      dma16(rb, voff, 0, slot + TSLOT_A + i * NLW * 1024);
      tox[i] += BKS;
      while (tox[i] >= cg.Wo) {
        tox[i] -= cg.Wo;
        if (++toy[i] == cg.Ho) {
          toy[i] = 0;
          ++timg[i];
        }
      }
    } else {
      dma16(rb, odd ? vb_o : vb_e, (int)((unsigned)s * b_sl + (unsigned)r16 * (b_sl >> 1)),
            slot + TSLOT_A + i * NLW * 1024);
    }
  };
  auto stage = [&](int s) {
#pragma unroll
    for (int o = 0; o < OPS; ++o) stage_op(s, o);
  };
  // the ops of one slice spread over the step's 4 MFMA groups
  auto stage_group = [&](int s, int grp) {
#pragma unroll
    for (int o = grp * OPS / 4; o < (grp + 1) * OPS / 4; ++o) stage_op(s, o);
  };

  // ---- transposed fragment reads: lane l (group g = l >> 4, e = l & 15, q = e >> 2, p = e & 3)
  // supplies, for read h, the address of token row 8g + 4h + q, columns c0 + 4p .. c0 + 4p + 3 of the
  // 16-column block; it receives column c0 + e of the 4 rows. Rows r0 and r0 + 4 have the same F (F
  // ignores row bit 2), so the read of row r0 + 4 is the read of row r0 plus the immediate 4 * TROW.
  const int g = lane >> 4, e = lane & 15, qq = e >> 2, pp = e & 3;
  const int r0 = 8 * g + qq;
  const int f0 = swz(r0);
  const int half8 = (pp & 1) * 8, hchunk = pp >> 1;
  auto toff = [&](int c) { return r0 * TROW + ((((c >> 3) ^ f0) + hchunk) << 4) + half8; };

  sx8 x[6];
  auto xfrag = [&](int s, int i) {  // A row block i of slice s
    const char* so = smem + (s & 3) * SLOT_BYTES;
    const int c = wm * 128 + 16 * i;
    return tr_frag(so + toff(c), so + toff(c) + 4 * TROW);
  };
  auto wfrag = [&](int s, int j) {  // B column block j of slice s
    const char* so = smem + (s & 3) * SLOT_BYTES + TSLOT_A;
    const int c = wn * 64 + 16 * j;
    return tr_frag(so + toff(c), so + toff(c) + 4 * TROW);
  };
  // part 0: x[0, 1], w[0, 1]; part 1: x[2, 3], w[2, 3]; part 2: x[4, 5], y[0, 1]
  auto load_part = [&](Frags& f, int s, int part) {
    x[2 * part] = xfrag(s, 2 * part);
    x[2 * part + 1] = xfrag(s, 2 * part + 1);
    if (part < 2) {
      f.w[2 * part] = wfrag(s, 2 * part);
      f.w[2 * part + 1] = wfrag(s, 2 * part + 1);
    } else {
      f.y[0] = xfrag(s, 6);
      f.y[1] = xfrag(s, 7);
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

  auto mma = [&](const Frags& f, auto I0, auto I1) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = decltype(I0)::value; i < decltype(I1)::value; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const sx8& xf = i < 6 ? x[i < 6 ? i : 0] : f.y[i >= 6 ? i - 6 : 0];
        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(f.w[j], xf, acc[i][j], 0, 0, 0);
      }
    __builtin_amdgcn_s_setprio(0);
  };
  using I0c = std::integral_constant<int, 0>;
  using I2c = std::integral_constant<int, 2>;
  using I4c = std::integral_constant<int, 4>;
  using I6c = std::integral_constant<int, 6>;
  using I8c = std::integral_constant<int, 8>;

  // one step: slice s in registers; make slice s + 1 visible (a loader's counted vmcnt leaves the two
  // slices behind it in flight), issue slice s + 4 into the slot of slice s, read slice s + 1 into fn,
  // MFMAs of slice s; the DMA ops and ds_reads interleave with the 4 MFMA groups
  auto step = [&](int s, Frags& fc, Frags& fn, auto ROLE, auto STAGE, auto PEND) {
    constexpr bool loader = decltype(ROLE)::value, st = decltype(STAGE)::value && loader;
    if constexpr (loader)
      wait_vm<decltype(PEND)::value>();  // own DMA of slice s + 1 retired; own ds_reads too
    else
      wait_lgkm0();  // compute-only waves: their ds_reads
    barrier();
    if constexpr (st) stage_group(s + 4, 0);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I0c{}, I2c{});
    __builtin_amdgcn_sched_barrier(0);
    load_part(fn, s + 1, 0);
    if constexpr (st) stage_group(s + 4, 1);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I2c{}, I4c{});
    __builtin_amdgcn_sched_barrier(0);
    load_part(fn, s + 1, 1);
    if constexpr (st) stage_group(s + 4, 2);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I4c{}, I6c{});
    __builtin_amdgcn_sched_barrier(0);
    load_part(fn, s + 1, 2);
    if constexpr (st) stage_group(s + 4, 3);
    __builtin_amdgcn_sched_barrier(0);
    mma(fc, I6c{}, I8c{});
  };

  using T = std::true_type;
  using F = std::false_type;
  using PS = std::integral_constant<int, 2 * OPS>;  // steady state: two staging steps after slice s + 1
  using PT1 = std::integral_constant<int, OPS>;
  using P0 = std::integral_constant<int, 0>;
  Frags f0r, f1r;
  auto run = [&](auto ROLE) {
    if constexpr (decltype(ROLE)::value) {
      stage(0);
      stage(1);
      stage(2);
      stage(3);
      wait_vm<3 * OPS>();  // slice 0 landed
    }
    barrier();
    load(f0r, 0);
    int s = 0;
#pragma unroll 1
    for (; s + 5 < nk; s += 2) {
      step(s, f0r, f1r, ROLE, T{}, PS{});
      step(s + 1, f1r, f0r, ROLE, T{}, PS{});
    }
    step(s, f0r, f1r, ROLE, F{}, PS{});
    step(s + 1, f1r, f0r, ROLE, F{}, PT1{});
    step(s + 2, f0r, f1r, ROLE, F{}, P0{});
    mma(f1r, I0c{}, I8c{});
  };
  if (NLW == 8 || wid < NLW)
    run(T{});
  else
    run(F{});

  // ---- fp32 partial: acc[i][j] = C[m][n .. n + 3], m = row block i + (lane & 15), n = column block j.
  // Ragged M (M % 256 = 128: the LM head's 50304 rows): the last row panel's lanes for columns past M
  // re-read the panel's last valid chunk (the clamp of cha_e / cha_o above), and those output rows are
  // not stored
  const int mrow = m0 + wm * 128 + (lane & 15);
  const int ncol = n0 + wn * 64 + 4 * (lane >> 4);
  float* cp = Cpart + (int64_t)split * M * N;
#pragma unroll
  for (int i = 0; i < 8; ++i)
    if (mrow + 16 * i < M) {
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (ncol + 16 * j < N) *(f32x4*)(cp + (int64_t)(mrow + 16 * i) * N + ncol + 16 * j) = acc[i][j];
    }
}

// out[i] (bf16) = (accumulate ? out[i] : 0) + sum_s part[s][i], 4 elements per thread
__global__ void __launch_bounds__(256) splitk_sum_kernel(const float* __restrict__ part, bf16* __restrict__ out,
                                                         int64_t n, int splits, int accumulate) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  if (i >= n) return;
  f32x4 a = *(const f32x4*)(part + i);
  for (int s = 1; s < splits; ++s) a += *(const f32x4*)(part + (int64_t)s * n + i);
  bf16x4 o = *(bf16x4*)(out + i);
  bf16x4 r;
#pragma unroll
  for (int t = 0; t < 4; ++t) r[t] = (bf16)((accumulate ? (float)o[t] : 0.f) + a[t]);
  *(bf16x4*)(out + i) = r;
}

}  // namespace gemm_wg
}  // namespace vcx

using namespace vcx;

using gemm_wg::ConvG;

bool vcx_gemm_wg_supported(int M, int N, int K, int splits) {
  if (!(M > 0 && N > 0 && M % 128 == 0 && N % gemm_wg::BN == 0 && K % 64 == 0 && splits >= 1 &&
        K / 192 >= splits))  // >= 3 blocks of 64 tokens per split (nk >= 6)
    return false;
  // a split's operand panels stay under 2 GB (32-bit buffer offsets, slice offsets in soffset)
  const int64_t tok = ((int64_t)(K / 64 + splits - 1) / splits) * 64;
  return tok * std::max(M, N) * 2 < (int64_t(1) << 31) - (int64_t(1) << 20);
}

// token-axis splits: about one round of workgroups over the CUs ((M/256)(N/256) tiles x S), with at least
// 768 tokens per split: each split writes a 256 KB fp32 partial per tile that splitk_sum reads back, so
// short splits move more partial bytes than operand bytes (ResNet-50 at 25k / 6k tokens: 64 / 16 splits of
// 392 tokens -> 32 / 8 of 784: config 3 8635-8656 vs 8556-8562 img/s, gpurun_out/c17; the GPT-2 shapes,
// 65536 tokens, keep their split counts). VCX_WG_TARGET: the workgroup count aimed at (default 256).
static int wg_target() {
  static const int t = [] {
    const char* e = std::getenv("VCX_WG_TARGET");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 256;
  }();
  return t;
}

int vcx_gemm_wg_splits(int M, int N, int K) {
  const int tiles = ((M + gemm_wg::BM - 1) / gemm_wg::BM) * ((N + gemm_wg::BN - 1) / gemm_wg::BN);
  if (tiles > wg_target()) {
    // more tiles than one round (the LM head: 591): 1..4 splits, the fewest rounds of workgroups per unit of
    // work -- ceil(tiles S / 256) / S -- among the counts whose split panels stay under 2 GB
    int best = 0;
    double best_cost = 1e30;
    for (int s = 1; s <= 4 && s <= K / 768; ++s) {
      const int64_t tok = ((int64_t)(K / 64 + s - 1) / s) * 64;
      if (tok * std::max(M, N) * 2 >= (int64_t(1) << 31) - (int64_t(1) << 20)) continue;
      const double cost = (double)((tiles * s + wg_target() - 1) / wg_target()) / s;
      if (cost < best_cost - 1e-9) best_cost = cost, best = s;
    }
    return best > 0 ? best : 4;
  }
  int s = wg_target() / (tiles > 0 ? tiles : 1);
  if (s < 1) s = 1;
  if (s > K / 768) s = K / 768;
  return s < 1 ? 1 : s;
}

// Cpart[splits, M, N] (fp32 workspace) = per-split A[K, M]^T . B[K, N]; then out (bf16 [M, N], row
// stride N) = (accumulate ? out : 0) + the sum of the partials. loaders: 8 (default) or 4 waves stage.
static void launch_wg(const void* A, const void* B, float* Cpart, void* out, int M, int N, int K, int lda, int ldb,
                      int splits, int accumulate, int loaders, ConvG cg, hipStream_t s) {
  using namespace gemm_wg;
  const int tilesN = (N + BN - 1) / BN, tiles = ((M + BM - 1) / BM) * tilesN;
  static const bool attrs = [] {
    for (const void* k : {(const void*)gemm_wg_kernel<4, false>, (const void*)gemm_wg_kernel<8, false>,
                          (const void*)gemm_wg_kernel<8, true>})
      (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    return true;
  }();
  (void)attrs;
  auto go = [&](auto kern) {
    hipLaunchKernelGGL(kern, dim3(tiles * splits), dim3(NT), LDS_BYTES, s, (const bf16*)A, (const bf16*)B, Cpart, M,
                       N, K, lda, ldb, tilesN, tiles, splits, cg);
  };
  if (cg.Cin > 0)
    go(gemm_wg_kernel<8, true>);
  else if (loaders == 4)
    go(gemm_wg_kernel<4, false>);
  else
    go(gemm_wg_kernel<8, false>);
  const int64_t n = (int64_t)M * N;
  hipLaunchKernelGGL(splitk_sum_kernel, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, s, Cpart, (bf16*)out, n,
                     splits, accumulate);
}

void vcx_gemm_wg(const void* A, const void* B, float* Cpart, void* out, int M, int N, int K, int lda, int ldb,
                 int splits, int accumulate, int loaders, hipStream_t s) {
  launch_wg(A, B, Cpart, out, M, N, K, lda, ldb, splits, accumulate, loaders, ConvG{0, 0, 0, 0, 0, 0, 0}, s);
}

// 3x3 convolution (pad 1) weight gradient: out[Cout, 9 Cin] (+)= dY[tokens, Cout]^T P(x), the channels-last
// weight layout; dy NHWC [imgs, Ho, Wo, Cout], x NHWC [imgs, H, W, Cin]; splits <= 0: vcx_gemm_wg_splits
bool vcx_gemm_wg_conv3x3_supported(int Cout, int Cin, int tokens, int64_t xbytes, int splits) {
  return Cout > 0 && Cin > 0 && Cout % 128 == 0 && Cin % 128 == 0 && tokens > 0 && tokens % 64 == 0 &&
         splits >= 1 && tokens / 192 >= splits && xbytes + 64 < (int64_t(1) << 31);
}

void vcx_gemm_wg_conv3x3(const void* dy, const void* x, float* Cpart, void* out, int Cout, int Cin, int imgs, int H,
                         int W, int stride, int splits, int accumulate, hipStream_t s) {
  const int Ho = (H - 1) / stride + 1, Wo = (W - 1) / stride + 1;
  const int64_t xbytes = (int64_t)imgs * H * W * Cin * 2;
  launch_wg(dy, x, Cpart, out, Cout, 9 * Cin, imgs * Ho * Wo, Cout, 0, splits, accumulate, 8,
            ConvG{H, W, Ho, Wo, Cin, stride, (int)xbytes}, s);
}
