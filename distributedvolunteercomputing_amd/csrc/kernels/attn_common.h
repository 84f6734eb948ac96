// Shared device helpers of the attention kernels (attention.hip: packed-QKV GPT-2 layout, head
// dim 64; attention_hm.hip: head-major GQA layout, head dim 64/128): MFMA wrappers, the
// XOR-swizzled LDS tile image and its row / transposed fragment reads, LDS-DMA tile loads, lane-half
// reductions, accumulator-tile stores and column sums. See attention.hip for the design notes.
#pragma once
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

}  // namespace vcx
