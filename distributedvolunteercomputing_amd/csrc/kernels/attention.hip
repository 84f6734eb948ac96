// Causal flash attention for head dim 64 on gfx950 (GPT-2 family), bf16 in/out, fp32 softmax.
//
// Layouts (no permute/copy kernels around attention):
//   qkv  : [B, T, 3, H, 64] bf16 — exactly the output of the fused QKV projection GEMM
//   o    : [B, T, H, 64]    bf16 — exactly the input of the output projection GEMM
//   lse  : [B, H, T]        fp32 — log2-domain row log-sum-exp saved for the backward
//   dqkv : [B, T, 3, H, 64] bf16 — written directly by the backward kernels (no torch.cat)
//
// MFMA structure (v_mfma_f32_32x32x16_bf16, wave64): the score tile is computed TRANSPOSED,
// S^T[key, query] = K . Q^T, so every lane owns one query column and holds 16 of its 32 key
// scores in registers (its partner lane l^32 holds the other 16): the softmax row statistics
// need one cross-lane exchange, and the bf16-converted P^T accumulator is directly the B
// operand of O^T += V^T . P^T (cdna guide §3 "accumulator tile as the next MFMA's operand").
// The A operand V^T is read from the row-major V tile in LDS with ds_read_b64_tr_b16, in the
// permuted key order that the accumulator layout implies.
//
// LDS tiles: unpadded [rows][64] bf16 images with an XOR swizzle (swz below) that keeps both the
// ds_read_b128 row reads and the ds_read_b64_tr_b16 transposed reads conflict-free. K/V (Q/dO)
// tiles are double-buffered and staged through registers (issue next tile's global loads before
// the MFMAs, write LDS after).
#include <type_traits>

#include "vcx_common.h"

namespace vcx {

typedef short sx8 __attribute__((ext_vector_type(8)));
typedef short sx4 __attribute__((ext_vector_type(4)));

constexpr int AD = 64;         // head dim
constexpr int A_BQ = 128;      // queries per block (4 waves x 32)
constexpr int A_BK = 64;       // keys per LDS tile
constexpr float LOG2E = 1.4426950408889634f;

using I0 = std::integral_constant<int, 0>;
using I1 = std::integral_constant<int, 1>;

__device__ __forceinline__ sx4 lds_tr_b64(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) sx4*)(p));
}

// v_max3_f32 without the canonicalising v_max_f32 the compiler puts in front of fmaxf on MFMA
// results (scores are never NaN here)
// CAUTION: hipcc pads hazards only around instructions it generates itself, never for an asm
// statement (guide §5.7 item 2). Reading an MFMA's D from inside asm without the MFMA->VALU wait
// states returns stale partial sums on some waves of some launches (seen as run-to-run 1-ulp
// output differences: a wrong running max only changes the rounding). Every max3 over raw score
// accumulators is therefore preceded by mfma_read_fence.
__device__ __forceinline__ float max3(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// 18 wait states (a 16-pass v_mfma_f32_32x32x16_bf16's D -> VALU read); the "+v" operands order
// this statement after both score MFMA chains and before the asm max3 that read them
__device__ __forceinline__ void mfma_read_fence(f32x16& a, f32x16& b) {
  asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 1" : "+v"(a), "+v"(b));
}

__device__ __forceinline__ f32x16 mfma32(sx8 a, sx8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ short bf16_bits(float f) {
  bf16 b = (bf16)f;
  return *(short*)&b;
}

// bf16 fragment times c, rounded back to bf16: the score scale (1/sqrt(D) * log2 e) is folded into
// the register-resident operand of S = Q K^T once per kernel instead of one v_fma per score (dQ
// kernel; the same change measured no faster in the forward, which then spills more, and slower in
// dK/dV, where the row constants come from LDS and their reads then precede the S MFMAs)
__device__ __forceinline__ sx8 prescale(sx8 v, float c) {
  sx8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const short sv = v[j];
    r[j] = bf16_bits((float)*(const bf16*)&sv * c);
  }
  return r;
}

__device__ __forceinline__ f32x16 splat16(float v) {
  f32x16 r;
#pragma unroll
  for (int i = 0; i < 16; ++i) r[i] = v;
  return r;
}

// XOR-swizzled [rows][64] bf16 LDS tile (no padding): 16-B chunk c of row r is stored at chunk
// c ^ g((r >> 1) & 7), g(k) = ((k & 1) << 2) | (k >> 1). Even and odd rows fall in opposite
// 128-B halves of the 256-B bank row; g is a bijection on 0..7 (16 consecutive rows of one
// chunk -> 16 distinct 4-bank slots: ds_read_b128 row reads conflict-free) and g(2m), g(2m+1)
// differ in bit 2 (the 4 rows x 4 chunks of a half-wave ds_read_b64_tr_b16 hit 64 distinct
// banks). One image serves both the row-operand reads and the transposed reads.
__device__ __forceinline__ int swz(int r, int chunk) {
  const int k = (r >> 1) & 7;
  return r * 64 + ((chunk ^ (((k & 1) << 2) | (k >> 1))) << 3);
}

__device__ __forceinline__ sx8 row_frag_swz(const bf16* tile, int row, int s, int h) {
  return *(const sx8*)(tile + swz(row, 2 * s + h));
}

__device__ __forceinline__ sx8 vt_frag_swz(const bf16* tile, int key0, int dtile, int s, int lane) {
  const int h = lane >> 5, g = lane >> 4, lig = lane & 15, p = lig & 3;
  const int chunk = dtile * 4 + (g & 1) * 2 + (p >> 1);
  const int rb = key0 + 16 * s + 4 * h + (lig >> 2);
  sx4 lo = lds_tr_b64(tile + swz(rb, chunk) + 4 * (p & 1));
  sx4 hi = lds_tr_b64(tile + swz(rb + 8, chunk) + 4 * (p & 1));
  return sx8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// Bijective XCD-aware block remap (cdna guide §5 T1): hardware block b runs on XCD group b % 8;
// give each group a CONTIGUOUS range of logical blocks so all query tiles of one (batch, head)
// share that XCD's L2 copy of K/V.
__device__ __forceinline__ int xcd_remap(int b, int nwg) {
  if (nwg < 8) return b;
  const int q = nwg / 8, r = nwg % 8, x = b % 8, i = b / 8;
  return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + i;
}

// value of lane l combined with lane l ^ 32 by ONE v_permlane32_swap (VALU, no LDS round trip;
// __shfl_xor(v, 32) lowers to ds_bpermute on gfx950, ~100+ cycles in the softmax's serial chain)
typedef int i32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float xhalf_max(float v) {
  const i32x2 r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return fmaxf(__int_as_float(r[0]), __int_as_float(r[1]));
}
__device__ __forceinline__ float xhalf_sum(float v) {
  const i32x2 r = __builtin_amdgcn_permlane32_swap(__float_as_int(v), __float_as_int(v), false, false);
  return __int_as_float(r[0]) + __int_as_float(r[1]);
}

// Column sums of a wave's accumulator tile for the fused QKV-bias gradient. v holds the 32 values
// of one lane (= one row; the two 32-lane halves hold different columns); each step exchanges
// half of the live registers with lane l ^ K (ds_swizzle, 32-lane groups) and adds, so the live
// set halves: 31 swizzles in all. Afterwards v[0] of lane c of a half = the sum over the half's
// 32 rows of register c.
template <int K>
__device__ __forceinline__ float swz_xor(float x) {
  return __int_as_float(__builtin_amdgcn_ds_swizzle(__float_as_int(x), (K << 10) | 0x1F));
}
template <int K>
__device__ __forceinline__ void fold_step(float (&v)[32], int col) {
  const bool hi = (col & K) != 0;
#pragma unroll
  for (int j = 0; j < K; ++j) {
    const float keep = hi ? v[j + K] : v[j];
    const float send = hi ? v[j] : v[j + K];
    v[j] = keep + swz_xor<K>(send);
  }
}
__device__ __forceinline__ float half_colsum32(float (&v)[32], int col) {
  fold_step<16>(v, col);
  fold_step<8>(v, col);
  fold_step<4>(v, col);
  fold_step<2>(v, col);
  fold_step<1>(v, col);
  return v[0];
}
// head-dim column of register c (0..31) of the pair of 32x32 accumulators (c < 16: first, d < 32)
// in the lane half h2: registers 4g + i hold d = 8g + 4 h2 + i
__device__ __forceinline__ int acc_pair_col(int c, int h2) { return (c & 16) * 2 + 8 * ((c & 15) >> 2) + 4 * h2 + (c & 3); }

// Stores a wave's 32-row x 64-column accumulator pair (a0: columns 0-31, a1: 32-63; lane = row
// `col`, registers 4g + i = column 8g + 4 h2 + i) times `mul` (per lane = per row) as bf16 rows of
// a row-major matrix (dst = row 0, row stride ld; rows >= nrows are skipped). staged: through a
// wave-private, chunk-swizzled 32 x 64 LDS image `img`, then 4 fully coalesced 16-B stores per lane
// (whole 128-B rows) instead of 8 half-row 8-B stores.
__device__ __forceinline__ void store_acc_tile(const f32x16& a0, const f32x16& a1, float mul, bf16* dst, int64_t ld,
                                               int nrows, bf16* img, bool staged, int lane) {
  const int col = lane & 31, h2 = lane >> 5;
  if (staged) {
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 v0 = {(bf16)(a0[4 * g] * mul), (bf16)(a0[4 * g + 1] * mul), (bf16)(a0[4 * g + 2] * mul),
                   (bf16)(a0[4 * g + 3] * mul)};
      bf16x4 v1 = {(bf16)(a1[4 * g] * mul), (bf16)(a1[4 * g + 1] * mul), (bf16)(a1[4 * g + 2] * mul),
                   (bf16)(a1[4 * g + 3] * mul)};
      *(bf16x4*)(img + col * AD + ((g ^ (col & 7)) << 3) + 4 * h2) = v0;
      *(bf16x4*)(img + col * AD + (((g + 4) ^ (col & 7)) << 3) + 4 * h2) = v1;
    }
    __builtin_amdgcn_wave_barrier();  // the wave reads back only its own image
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int r = i * 8 + (lane >> 3), c = lane & 7;
      const bf16x8 v = *(const bf16x8*)(img + r * AD + ((c ^ (r & 7)) << 3));
      if (r < nrows) *(bf16x8*)(dst + r * ld + c * 8) = v;
    }
  } else if (col < nrows) {
    bf16* row = dst + col * ld;
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 8 * g + 4 * h2;
      bf16x4 v0 = {(bf16)(a0[4 * g] * mul), (bf16)(a0[4 * g + 1] * mul), (bf16)(a0[4 * g + 2] * mul),
                   (bf16)(a0[4 * g + 3] * mul)};
      bf16x4 v1 = {(bf16)(a1[4 * g] * mul), (bf16)(a1[4 * g + 1] * mul), (bf16)(a1[4 * g + 2] * mul),
                   (bf16)(a1[4 * g + 3] * mul)};
      *(bf16x4*)(row + d) = v0;
      *(bf16x4*)(row + 32 + d) = v1;
    }
  }
}

// LDS-DMA of a 64-row x 64-column bf16 tile — rows r0 .. r0+63 of a row-major matrix with row
// stride `ld` elements, row indices clamped to rmax — into the XOR-swizzled image `img` (swz
// layout). Each of the 4 waves moves two 1-KB pieces with global_load_lds_dwordx4; the DMA writes a
// wave-instruction's 64 x 16 B linearly, so the swizzle is applied to each lane's SOURCE address:
// LDS slot p (row p/8, stored chunk p%8) receives global chunk (p%8) ^ g(row).
__device__ __forceinline__ void dma_tile_swz(const bf16* g, int64_t ld, int r0, int rmax, bf16* img, int w,
                                             int lane) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int piece = w * 2 + i;  // wave-uniform
    const int p = piece * 64 + lane;
    const int r = p >> 3, k = (r >> 1) & 7;
    const int chunk = (p & 7) ^ (((k & 1) << 2) | (k >> 1));
    const int row = min(r0 + r, rmax);
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(g + (int64_t)row * ld + chunk * 8),
                                     (__attribute__((address_space(3))) void*)(img + piece * 512), 16, 0, 0);
  }
}

// ============================================================================ forward
// Forward, occupancy-templated: the same tile algorithm with both K and V in XOR-swizzled
// UNPADDED images (2 buffers x (8 + 8) KB = 32 KB per block, vs 42 KB padded) and the row max /
// row sum combined across the lane halves by v_permlane32_swap. With WPE = 4 the kernel is held
// to 128 VGPRs so FOUR blocks (16 waves, 4 per SIMD) share a CU: the per-tile chain (K reads ->
// S MFMAs -> max -> exp -> P -> V^T reads -> PV MFMAs -> barrier) is serial inside a wave, so the
// SIMD needs more waves to overlap one wave's softmax with another's MFMAs.
//
// DMA = true stages K/V with LDS-DMA (global_load_lds_dwordx4: no staging registers, no ds_write
// pass; the swizzle moves to the per-lane SOURCE address since the DMA writes each wave's 1-KB
// piece linearly) instead of global_load -> VGPR -> ds_write.
template <int WPE, bool DMA>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
attn_fwd_d64_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, float* __restrict__ lse, int B, int T, int H,
                    float scale_log2, int staged_epi) {  // staged_epi: store_acc_tile
  // one shared object per buffer, so the compiler can tell that the LDS-DMA into one buffer
  // does not alias the reads of the other (else it waits vmcnt(0) before every V^T read)
  __shared__ __attribute__((aligned(16))) bf16 sKV0[2][A_BK * AD];  // [K | V], swizzled (swz)
  __shared__ __attribute__((aligned(16))) bf16 sKV1[2][A_BK * AD];
#define sK_(b) ((b) ? &sKV1[0][0] : &sKV0[0][0])
#define sV_(b) ((b) ? &sKV1[1][0] : &sKV0[1][0])
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h2 = lane >> 5, col = lane & 31;
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = nqt - 1 - (lb % nqt);  // heaviest (last) query tiles first
  const int bh = lb / nqt;
  const int b = bh / H, hh = bh % H;
  const int64_t tok = 3ll * H * AD;
  const bf16* base = qkv + (int64_t)b * T * tok + hh * AD;
  const bf16* Kg = base + H * AD;
  const bf16* Vg = base + 2 * H * AD;
  const int q0 = qt * A_BQ;
  const int qw = q0 + w * 32;
  const int q = qw + col;
  const int qc = min(q, T - 1);
  sx8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *(const sx8*)(base + (int64_t)qc * tok + 16 * s + 8 * h2);
  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  const int kend = min(T, q0 + A_BQ);
  const int nkt = (kend + A_BK - 1) / A_BK;
  sx8 rk[2], rv[2];
  // register staging: load tile kt into rk/rv (sstore writes them to buffer buf later);
  // DMA staging: tile kt goes straight into buffer buf (sstore is a no-op)
  auto gload = [&](int kt, int buf) {
    if constexpr (DMA) {
      dma_tile_swz(Kg, tok, kt * A_BK, T - 1, sK_(buf), w, lane);
      dma_tile_swz(Vg, tok, kt * A_BK, T - 1, sV_(buf), w, lane);
    } else {
      (void)buf;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, r = e >> 3, c = (e & 7) * 8;
        const int key = min(kt * A_BK + r, T - 1);
        rk[i] = *(const sx8*)(Kg + (int64_t)key * tok + c);
        rv[i] = *(const sx8*)(Vg + (int64_t)key * tok + c);
      }
    }
  };
  auto sstore = [&](int buf) {
    if constexpr (!DMA) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, r = e >> 3;
        *(sx8*)(sK_(buf) + swz(r, e & 7)) = rk[i];
        *(sx8*)(sV_(buf) + swz(r, e & 7)) = rv[i];
      }
    }
  };
  auto tile = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const int kb = kt * A_BK;
    if (MASK && kb > qw + 31) return;
    f32x16 s0 = {}, s1 = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma32(row_frag_swz(sK_(cur), col, s, h2), qf[s], s0);
      s1 = mfma32(row_frag_swz(sK_(cur), 32 + col, s, h2), qf[s], s1);
    }
    mfma_read_fence(s0, s1);
    if (MASK) {
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * h2;
        s0[r] = key > q ? -INFINITY : s0[r];
        s1[r] = key + 32 > q ? -INFINITY : s1[r];
      }
    }
    float mx0 = max3(s0[0], s0[1], s1[0]), mx1 = max3(s1[1], s0[2], s1[2]);
#pragma unroll
    for (int r = 3; r < 15; r += 2) {
      mx0 = max3(mx0, s0[r], s1[r]);
      mx1 = max3(mx1, s0[r + 1], s1[r + 1]);
    }
    const float mx = xhalf_max(max3(mx0, mx1, fmaxf(s0[15], s1[15]))) * scale_log2;
    if (!__all(mx - m <= 8.f)) {  // deferred rescale (T13), threshold 2^8
      const float mnew = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      l *= alpha;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        o0[r] *= alpha;
        o1[r] *= alpha;
      }
      m = mnew;
    }
    const float mneg = -m;
    float ps0 = 0.f, ps1 = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float p0 = __builtin_amdgcn_exp2f(fmaf(s0[r], scale_log2, mneg));
      const float p1 = __builtin_amdgcn_exp2f(fmaf(s1[r], scale_log2, mneg));
      s0[r] = p0;
      s1[r] = p1;
      ps0 += p0;
      ps1 += p1;
    }
    l += xhalf_sum(ps0 + ps1);
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f32x16& sp = (s < 2) ? s0 : s1;
      sx8 pb;
#pragma unroll
      for (int j = 0; j < 8; ++j) pb[j] = bf16_bits(sp[8 * (s & 1) + j]);
      o0 = mfma32(vt_frag_swz(sV_(cur), (s >> 1) * 32, 0, s & 1, lane), pb, o0);
      o1 = mfma32(vt_frag_swz(sV_(cur), (s >> 1) * 32, 1, s & 1, lane), pb, o1);
    }
  };
  gload(0, 0);
  sstore(0);
  __syncthreads();
  // Retire EVERY outstanding global load (the per-lane Q/dO/K/V fragments loaded at kernel entry
  // included) before the tile loop. hipcc issues those fragment loads after the first tile's
  // staging loads and does not wait for them in the prologue; the waitcnt pass then merges that
  // pending state into the loop header and makes every iteration wait vmcnt(3..0) for its own
  // next-tile prefetch before the first MFMA that reads a fragment register — serialising the
  // prefetch with the compute (seen in the forward's ISA). The builtin (not inline asm: the
  // waitcnt pass cannot see into an asm statement) is vmcnt(0) with expcnt/lgkmcnt at their
  // maxima in the gfx9 encoding: vmcnt[3:0] = 0, expcnt[6:4] = 7, lgkmcnt[11:8] = 15.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const int kdiag = q0 / A_BK;
  auto step = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (kt + 1 < nkt) gload(kt + 1, cur ^ 1);
    tile(kt, cur_c, mask_c);
    if (kt + 1 < nkt) sstore(cur ^ 1);
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < kdiag; kt += 2) {
    step(kt, I0{}, std::false_type{});
    step(kt + 1, I1{}, std::false_type{});
  }
  if (kt < kdiag) step(kt++, I0{}, std::false_type{});
  for (; kt < nkt; ++kt) {
    if (kt & 1)
      step(kt, I1{}, std::true_type{});
    else
      step(kt, I0{}, std::true_type{});
  }
  const float inv = 1.f / l;
  store_acc_tile(o0, o1, inv, out + ((int64_t)b * T + qw) * H * AD + hh * AD, (int64_t)H * AD, T - qw,
                 &sKV0[0][0] + w * 32 * AD, staged_epi, lane);
  if (q < T && h2 == 0) lse[((int64_t)b * H + hh) * T + q] = m + __log2f(l);
#undef sK_
#undef sV_
}

// ============================================================================ backward
// dQ (query-parallel; same tiling as the forward): per 32-key sub-tile
//   S^T = K Q^T, P^T = exp2(S^T c - lse), dP^T = V dO^T, dS^T = P^T (dP^T - delta),
//   dQ^T += K^T dS^T  (A = K^T through ds_read_b64_tr_b16, B = dS^T from the accumulator)
template <int WPE, bool DMA>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) attn_bwd_dq_d64_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout,
                                                               const bf16* __restrict__ out, const float* __restrict__ lse,
                                                               float* __restrict__ delta, bf16* __restrict__ dqkv,
                                                               float* __restrict__ bpart,
                                                               int B, int T, int H, float scale, float scale_log2,
                                                               int staged_epi) {
  // one shared object per buffer (see the forward): [K | V] tiles, swizzled (swz)
  __shared__ __attribute__((aligned(16))) bf16 sKV0[2][A_BK * AD];
  __shared__ __attribute__((aligned(16))) bf16 sKV1[2][A_BK * AD];
#define sK_(b) ((b) ? &sKV1[0][0] : &sKV0[0][0])
#define sV_(b) ((b) ? &sKV1[1][0] : &sKV0[1][0])
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h2 = lane >> 5, col = lane & 31;
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = nqt - 1 - (lb % nqt);
  const int bh = lb / nqt;
  const int b = bh / H, hh = bh % H;
  const int64_t tok = 3ll * H * AD;
  const bf16* base = qkv + (int64_t)b * T * tok + hh * AD;
  const bf16* Kg = base + H * AD;
  const bf16* Vg = base + 2 * H * AD;
  const int64_t otok = (int64_t)H * AD;
  const bf16* dOb = dout + (int64_t)b * T * otok + hh * AD;
  const int q0 = qt * A_BQ, qw = q0 + w * 32, q = qw + col, qc = min(q, T - 1);
  sx8 qf[4], df[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    qf[s] = *(const sx8*)(base + (int64_t)qc * tok + 16 * s + 8 * h2);
    df[s] = *(const sx8*)(dOb + (int64_t)qc * otok + 16 * s + 8 * h2);
  }
  const float nlq = -lse[((int64_t)b * H + hh) * T + qc];
  // row constants as the initial accumulators: S' = (c Q) K^T - lse and dP' = dO V^T - delta,
  // so p = exp2(S') and dS = p * dP' need no per-score fma / subtract
  const f32x16 lq16 = splat16(nlq);
  // delta[q] = sum_d dO[q, d] * O[q, d], computed here from the dO fragments already in registers
  // (this lane holds 32 of the 64 d, its partner lane l ^ 32 the rest) instead of by a separate
  // kernel; written out for the dK/dV kernel, which runs after this one
  float dq_delta;
  {
    const bf16* Ob = out + ((int64_t)b * T + qc) * otok + hh * AD;
    float acc = 0.f;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const sx8 ov = *(const sx8*)(Ob + 16 * s + 8 * h2);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const short ob = ov[j], db = df[s][j];
        acc = fmaf((float)*(const bf16*)&ob, (float)*(const bf16*)&db, acc);
      }
    }
    dq_delta = xhalf_sum(acc);
    if (h2 == 0 && q < T) delta[((int64_t)b * H + hh) * T + q] = dq_delta;
  }
  const f32x16 dl16 = splat16(-dq_delta);
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = prescale(qf[s], scale_log2);
  f32x16 a0 = {}, a1 = {};
  const int kend = min(T, q0 + A_BQ);
  const int nkt = (kend + A_BK - 1) / A_BK;
  sx8 rk[2], rv[2];
  auto gload = [&](int kt, int buf) {
    if constexpr (DMA) {
      dma_tile_swz(Kg, tok, kt * A_BK, T - 1, sK_(buf), w, lane);
      dma_tile_swz(Vg, tok, kt * A_BK, T - 1, sV_(buf), w, lane);
    } else {
      (void)buf;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, r = e >> 3, c = (e & 7) * 8;
        const int key = min(kt * A_BK + r, T - 1);
        rk[i] = *(const sx8*)(Kg + (int64_t)key * tok + c);
        rv[i] = *(const sx8*)(Vg + (int64_t)key * tok + c);
      }
    }
  };
  auto sstore = [&](int buf) {
    if constexpr (!DMA) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, r = e >> 3;
        *(sx8*)(sK_(buf) + swz(r, e & 7)) = rk[i];
        *(sx8*)(sV_(buf) + swz(r, e & 7)) = rv[i];
      }
    }
  };
  // one 64-key tile (two 32-key sub-tiles); MASK only on the tiles crossing the diagonal
  auto tile = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;  // LDS buffer: compile-time -> immediate offsets
    constexpr bool MASK = decltype(mask_c)::value;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = kt * A_BK + sub * 32;
      if (MASK && kb > qw + 31) continue;
      f32x16 st = lq16, dp = dl16;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(row_frag_swz(sK_(cur), sub * 32 + col, s, h2), qf[s], st);
        dp = mfma32(row_frag_swz(sV_(cur), sub * 32 + col, s, h2), df[s], dp);
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __builtin_amdgcn_exp2f(st[r]);
        if (MASK) {
          const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * h2;
          p = key > q ? 0.f : p;
        }
        st[r] = p * dp[r];  // dS^T
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        sx8 db;
#pragma unroll
        for (int j = 0; j < 8; ++j) db[j] = bf16_bits(st[8 * s + j]);
        a0 = mfma32(vt_frag_swz(sK_(cur), sub * 32, 0, s, lane), db, a0);
        a1 = mfma32(vt_frag_swz(sK_(cur), sub * 32, 1, s, lane), db, a1);
      }
    }
  };
  gload(0, 0);
  sstore(0);
  __syncthreads();
  // Retire EVERY outstanding global load (the per-lane Q/dO/K/V fragments loaded at kernel entry
  // included) before the tile loop. hipcc issues those fragment loads after the first tile's
  // staging loads and does not wait for them in the prologue; the waitcnt pass then merges that
  // pending state into the loop header and makes every iteration wait vmcnt(3..0) for its own
  // next-tile prefetch before the first MFMA that reads a fragment register — serialising the
  // prefetch with the compute (seen in the forward's ISA). The builtin (not inline asm: the
  // waitcnt pass cannot see into an asm statement) is vmcnt(0) with expcnt/lgkmcnt at their
  // maxima in the gfx9 encoding: vmcnt[3:0] = 0, expcnt[6:4] = 7, lgkmcnt[11:8] = 15.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const int kdiag = q0 / A_BK;
  auto step = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (kt + 1 < nkt) gload(kt + 1, cur ^ 1);
    tile(kt, cur_c, mask_c);
    if (kt + 1 < nkt) sstore(cur ^ 1);
    __syncthreads();
  };
  int kt = 0;
  for (; kt + 1 < kdiag; kt += 2) {  // unrolled by two so the LDS buffer is a constant
    step(kt, I0{}, std::false_type{});
    step(kt + 1, I1{}, std::false_type{});
  }
  if (kt < kdiag) step(kt++, I0{}, std::false_type{});
  for (; kt < nkt; ++kt) {  // the (at most two) diagonal tiles
    if (kt & 1)
      step(kt, I1{}, std::true_type{});
    else
      step(kt, I0{}, std::true_type{});
  }
  store_acc_tile(a0, a1, scale, dqkv + ((int64_t)b * T + qw) * tok + hh * AD, tok, T - qw,  // slot 0 = dQ
                 &sKV0[0][0] + w * 32 * AD, staged_epi, lane);
  if (bpart) {  // column sums of this block's dQ rows: one partial row of the QKV bias gradient
    float v[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v[r] = q < T ? a0[r] * scale : 0.f;
      v[16 + r] = q < T ? a1[r] * scale : 0.f;
    }
    const float cs = half_colsum32(v, col);
    float* red = (float*)&sKV1[0][0];  // the K/V tiles are dead after the loop (sKV0 holds the dQ images)
    red[w * AD + acc_pair_col(col, h2)] = cs;
    __syncthreads();
    if (tid < AD)
      bpart[((int64_t)b * nqt + qt) * 3 * H * AD + hh * AD + tid] =
          (red[tid] + red[AD + tid]) + (red[2 * AD + tid] + red[3 * AD + tid]);
  }
#undef sK_
#undef sV_
}

// dK, dV (key-parallel, "key on the lane"): per 32-query sub-tile
//   S = Q K^T, P = exp2(S c - lse[q]), dP = dO V^T, dS = P (dP - delta[q]),
//   dV^T += dO^T P,  dK^T += Q^T dS   (A operands through ds_read_b64_tr_b16 on the Q/dO tiles,
//   B operands = the bf16-converted accumulators; the keys stay on the lanes throughout)
constexpr int B_BQ = 64;  // queries per LDS tile

template <int WPE, bool DMA>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) attn_bwd_dkdv_d64_kernel(const bf16* __restrict__ qkv,
                                                                 const bf16* __restrict__ dout,
                                                                 const float* __restrict__ lse,
                                                                 const float* __restrict__ delta,
                                                                 bf16* __restrict__ dqkv, float* __restrict__ bpart,
                                                                 int B, int T, int H, float scale, float scale_log2,
                                                                 int staged_epi) {
  // one shared object per buffer (see the forward): [Q | dO] tiles, swizzled (swz)
  __shared__ __attribute__((aligned(16))) bf16 sQD0[2][B_BQ * AD];
  __shared__ __attribute__((aligned(16))) bf16 sQD1[2][B_BQ * AD];
#define sQ_(b) ((b) ? &sQD1[0][0] : &sQD0[0][0])
#define sD_(b) ((b) ? &sQD1[1][0] : &sQD0[1][0])
  __shared__ __attribute__((aligned(16))) float sL[2][B_BQ];
  __shared__ __attribute__((aligned(16))) float sDel[2][B_BQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h2 = lane >> 5, col = lane & 31;
  const int nkb = (T + 127) / 128;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int kbi = lb % nkb;  // light (late) key blocks last
  const int bh = lb / nkb;
  const int b = bh / H, hh = bh % H;
  const int64_t tok = 3ll * H * AD;
  const bf16* base = qkv + (int64_t)b * T * tok + hh * AD;
  const int64_t otok = (int64_t)H * AD;
  const bf16* dOb = dout + (int64_t)b * T * otok + hh * AD;
  const float* lrow = lse + ((int64_t)b * H + hh) * T;
  const float* drow = delta + ((int64_t)b * H + hh) * T;
  const int k0 = kbi * 128, kw = k0 + w * 32, key = kw + col, kc = min(key, T - 1);
  sx8 kf[4], vf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    kf[s] = *(const sx8*)(base + H * AD + (int64_t)kc * tok + 16 * s + 8 * h2);
    vf[s] = *(const sx8*)(base + 2 * H * AD + (int64_t)kc * tok + 16 * s + 8 * h2);
  }
  f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
  const int qstart = k0 / B_BQ;  // first query tile that can see these keys
  const int nqt = (T + B_BQ - 1) / B_BQ;
  sx8 rq[2], rd[2];
  float rl = 0.f, rdl = 0.f;
  auto gload = [&](int qt, int buf) {
    if constexpr (DMA) {
      dma_tile_swz(base, tok, qt * B_BQ, T - 1, sQ_(buf), w, lane);
      dma_tile_swz(dOb, otok, qt * B_BQ, T - 1, sD_(buf), w, lane);
    } else {
      (void)buf;
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, r = e >> 3, c = (e & 7) * 8;
        const int qq = min(qt * B_BQ + r, T - 1);
        rq[i] = *(const sx8*)(base + (int64_t)qq * tok + c);
        rd[i] = *(const sx8*)(dOb + (int64_t)qq * otok + c);
      }
    }
    if (tid < B_BQ) {  // -lse (so P = exp2(S c + nl)); -inf for rows past T: their P is 0
      const int qq = qt * B_BQ + tid;
      rl = qq < T ? -lrow[qq] : -INFINITY;
      rdl = drow[min(qq, T - 1)];
    }
  };
  auto sstore = [&](int buf) {
    if constexpr (!DMA) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int e = tid + i * 256, r = e >> 3;
        *(sx8*)(sQ_(buf) + swz(r, e & 7)) = rq[i];
        *(sx8*)(sD_(buf) + swz(r, e & 7)) = rd[i];
      }
    }
    if (tid < B_BQ) {
      sL[buf][tid] = rl;
      sDel[buf][tid] = rdl;
    }
  };
  // one 64-query tile (two 32-query sub-tiles); MASK only on the two tiles that cross this
  // block's diagonal. Rows past T carry -inf in sL (P = 0) and keys past T are never stored.
  auto tile = [&](int qt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qb = qt * B_BQ + sub * 32;
      if (MASK && qb + 31 < kw) continue;  // every query before this wave's first key
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(row_frag_swz(sQ_(cur), sub * 32 + col, s, h2), kf[s], st);
        dp = mfma32(row_frag_swz(sD_(cur), sub * 32 + col, s, h2), vf[s], dp);
      }
      f32x16 pp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        // rows 8g + 4h + (0..3) of S are 4 consecutive queries: one 16-B LDS read each
        const f32x4 lv = *(const f32x4*)(&sL[cur][sub * 32 + 8 * g + 4 * h2]);
        const f32x4 dv = *(const f32x4*)(&sDel[cur][sub * 32 + 8 * g + 4 * h2]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          float p = __builtin_amdgcn_exp2f(fmaf(st[r], scale_log2, lv[i]));
          if (MASK) {
            const int qq = qb + 8 * g + 4 * h2 + i;
            p = key > qq ? 0.f : p;
          }
          pp[r] = p;
          st[r] = p * (dp[r] - dv[i]);  // dS
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        sx8 pb, sb;
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          pb[j] = bf16_bits(pp[8 * s + j]);
          sb[j] = bf16_bits(st[8 * s + j]);
        }
        dv0 = mfma32(vt_frag_swz(sD_(cur), sub * 32, 0, s, lane), pb, dv0);
        dv1 = mfma32(vt_frag_swz(sD_(cur), sub * 32, 1, s, lane), pb, dv1);
        dk0 = mfma32(vt_frag_swz(sQ_(cur), sub * 32, 0, s, lane), sb, dk0);
        dk1 = mfma32(vt_frag_swz(sQ_(cur), sub * 32, 1, s, lane), sb, dk1);
      }
    }
  };
  gload(qstart, 0);
  sstore(0);
  __syncthreads();
  // Retire EVERY outstanding global load (the per-lane Q/dO/K/V fragments loaded at kernel entry
  // included) before the tile loop. hipcc issues those fragment loads after the first tile's
  // staging loads and does not wait for them in the prologue; the waitcnt pass then merges that
  // pending state into the loop header and makes every iteration wait vmcnt(3..0) for its own
  // next-tile prefetch before the first MFMA that reads a fragment register — serialising the
  // prefetch with the compute (seen in the forward's ISA). The builtin (not inline asm: the
  // waitcnt pass cannot see into an asm statement) is vmcnt(0) with expcnt/lgkmcnt at their
  // maxima in the gfx9 encoding: vmcnt[3:0] = 0, expcnt[6:4] = 7, lgkmcnt[11:8] = 15.
  __builtin_amdgcn_s_waitcnt(0x0F70);
  auto step = [&](int qt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (qt + 1 < nqt) gload(qt + 1, cur ^ 1);
    tile(qt, cur_c, mask_c);
    if (qt + 1 < nqt) sstore(cur ^ 1);
    __syncthreads();
  };
  // queries k0 .. k0+127 (tiles qstart, qstart+1) cross the diagonal; later tiles are unmasked
  step(qstart, I0{}, std::true_type{});
  if (qstart + 1 < nqt) step(qstart + 1, I1{}, std::true_type{});
  int qt = qstart + 2;
  for (; qt + 1 < nqt; qt += 2) {  // unrolled by two so the LDS buffer is a constant
    step(qt, I0{}, std::false_type{});
    step(qt + 1, I1{}, std::false_type{});
  }
  if (qt < nqt) step(qt, I0{}, std::false_type{});
  if (bpart) {  // column sums of this block's dK and dV rows: slots 1 and 2 of a QKV-bias partial row
    float* red = (float*)&sQD0[0][0];  // the Q/dO tiles are dead after the last barrier of the loop
    float v[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v[r] = key < T ? dk0[r] * scale : 0.f;
      v[16 + r] = key < T ? dk1[r] * scale : 0.f;
    }
    red[w * AD + acc_pair_col(col, h2)] = half_colsum32(v, col);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v[r] = key < T ? dv0[r] : 0.f;
      v[16 + r] = key < T ? dv1[r] : 0.f;
    }
    red[4 * AD + w * AD + acc_pair_col(col, h2)] = half_colsum32(v, col);
    __syncthreads();
    if (tid < 2 * AD) {
      const int sl = tid >> 6, d = tid & 63;
      const float* rr = red + sl * 4 * AD;
      bpart[((int64_t)b * nkb + kbi) * 3 * H * AD + (1 + sl) * H * AD + hh * AD + d] =
          (rr[d] + rr[AD + d]) + (rr[2 * AD + d] + rr[3 * AD + d]);
    }
    __syncthreads();  // red is overwritten by the dK images below
  }
  bf16* dk_row0 = dqkv + ((int64_t)b * T + kw) * tok + H * AD + hh * AD;  // slot 1 = dK, slot 2 = dV
  store_acc_tile(dk0, dk1, scale, dk_row0, tok, T - kw, &sQD0[0][0] + w * 32 * AD, staged_epi, lane);
  store_acc_tile(dv0, dv1, 1.f, dk_row0 + H * AD, tok, T - kw, &sQD1[0][0] + w * 32 * AD, staged_epi, lane);
#undef sQ_
#undef sD_
}

}  // namespace vcx

using namespace vcx;

// Forward default: LDS-DMA staging at 3 waves per SIMD. Measured at the GPT-2 bench shape
// (B=64 H=12 T=1024, one process, interleaved rounds; scripts/attn_variants.py): 0.211 ms, vs
// 0.223 DMA at 2 waves/SIMD, 0.237 register staging at 2 and 0.266 register staging at 3 (spills).
// Backward kernels: 2 waves per SIMD (at 3-4 they spill: dq 0.87-1.25 ms vs 0.64 for the pair);
// dQ with LDS-DMA staging (264 vs 275 us), dK/dV with register staging (381 vs 383 us: the DMA
// build of that kernel hits the 256-VGPR cap and spills).
static int g_fwd_wpe = 3, g_fwd_dma = 1, g_bwd_dma = 1;  // g_bwd_dma bit 0: dQ kernel, bit 1: dK/dV kernel
// output tiles (O, dQ, dK, dV): 1 = staged through LDS, whole-row 16-B stores; 0 = per-lane half-row
// stores. Bench shape, same box (profiles/r1_attn_variants.log): backward 0.589 vs 0.614 ms, forward
// within noise (0.201-0.212 vs 0.206-0.208)
static int g_stage_epi = 1;

void vcx_attn_set_variant(int fwd_wpe, int fwd_dma, int bwd_dma, int stage_epi) {
  if (fwd_wpe == 2 || fwd_wpe == 3) g_fwd_wpe = fwd_wpe;
  if (fwd_dma == 0 || fwd_dma == 1) g_fwd_dma = fwd_dma;
  if (bwd_dma >= 0 && bwd_dma <= 3) g_bwd_dma = bwd_dma;
  if (stage_epi == 0 || stage_epi == 1) g_stage_epi = stage_epi;
}

int vcx_attn_bias_partials(int B, int T) { return B * ((T + 127) / 128); }

void vcx_attn_bwd_d64(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv,
                      float* bias_part, int B, int T, int H, float scale, hipStream_t s) {
  // dQ first: it also computes delta = rowsum(dO * O) for the dK/dV kernel
  const int nkb = (T + 127) / 128;
  const int nqt = (T + A_BQ - 1) / A_BQ;
  if (g_bwd_dma & 1)
    hipLaunchKernelGGL((attn_bwd_dq_d64_kernel<2, true>), dim3(B * H * nqt), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, (const bf16*)out, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale,
                       scale * LOG2E, g_stage_epi);
  else
    hipLaunchKernelGGL((attn_bwd_dq_d64_kernel<2, false>), dim3(B * H * nqt), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, (const bf16*)out, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale,
                       scale * LOG2E, g_stage_epi);
  if (g_bwd_dma & 2)
    hipLaunchKernelGGL((attn_bwd_dkdv_d64_kernel<2, true>), dim3(B * H * nkb), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale, scale * LOG2E,
                       g_stage_epi);
  else
    hipLaunchKernelGGL((attn_bwd_dkdv_d64_kernel<2, false>), dim3(B * H * nkb), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale, scale * LOG2E,
                       g_stage_epi);
}

void vcx_attn_fwd_d64(const void* qkv, void* out, float* lse, int B, int T, int H, float scale, hipStream_t s) {
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const dim3 g(B * H * nqt);
#define VCX_FWD(W, D)                                                                                      \
  hipLaunchKernelGGL((attn_fwd_d64_kernel<W, D>), g, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out, lse, B, T, H, \
                     scale * LOG2E, g_stage_epi)
  if (g_fwd_dma) {
    if (g_fwd_wpe == 2) VCX_FWD(2, true); else VCX_FWD(3, true);
  } else {
    if (g_fwd_wpe == 2) VCX_FWD(2, false); else VCX_FWD(3, false);
  }
#undef VCX_FWD
}
