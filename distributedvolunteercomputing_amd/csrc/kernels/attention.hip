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
#include <cstdio>
#include <cstdlib>

#include "attn_common.h"

namespace vcx {

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

// ---------------------------------------------------------------------------- forward, 3-slot ring
// The same tile algorithm with the K/V staging of gemm_wg: a 3-slot LDS ring
// (3 x 16 KB per block; three blocks per CU at 3 waves per SIMD = 144 KB), tile kt + 2 issued while
// tile kt computes, LDS-DMA as inline asm (invisible to hipcc's waitcnt pass, so it inserts no
// vmcnt(0) drain of its own), a COUNTED s_waitcnt that leaves the next tile's 4 pieces in flight
// across the raw s_barrier (the two-buffer kernel above drains every load at every tile: one
// vmcnt(0) per K/V tile in its ISA).
namespace ring {

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// buffer resource over [base, base + bytes): wave-uniform (SGPRs), 32-bit per-lane offsets
__device__ __forceinline__ u32x4 desc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  return u32x4{(unsigned)a, (unsigned)(a >> 32) & 0xffffu, bytes, 0x00020000u};
}

// one 1-KB LDS-DMA piece (16 B per lane to lds + 16 lane); M0 = LDS byte address; `s_nop 0`: M0 -> DMA hazard
__device__ __forceinline__ void dma16(u32x4 d, int voff, const bf16* lds) {
  const unsigned m0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) bf16*)lds;
  asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(d), "{m0}"(m0) : "memory");
}

// s_waitcnt vmcnt(N) lgkmcnt(0)
template <int N>
__device__ __forceinline__ void wait_vm() {
  static_assert(N >= 0 && N < 16, "vmcnt field");
  __builtin_amdgcn_s_waitcnt(0x0070 | N);
}
__device__ __forceinline__ void barrier() { asm volatile("s_barrier" ::: "memory"); }

constexpr int SLOT = 2 * A_BK * AD;  // elements: K tile then V tile (16 KB)

}  // namespace ring

template <int WPE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE)))
attn_fwd_d64_ring_kernel(const bf16* __restrict__ qkv, bf16* __restrict__ out, float* __restrict__ lse, int B, int T,
                         int H, float scale_log2, int staged_epi) {
  using namespace ring;
  __shared__ __attribute__((aligned(16))) bf16 sm[3 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, h2 = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = nqt - 1 - (lb % nqt);  // heaviest (last) query tiles first
  const int bh = lb / nqt;
  const int b = bh / H, hh = bh % H;
  const int64_t tok = 3ll * H * AD;
  const bf16* base = qkv + (int64_t)b * T * tok + hh * AD;
  const int q0 = qt * A_BQ;
  const int qw = q0 + w * 32;
  const int q = qw + col;
  const int qc = min(q, T - 1);
  sx8 qf[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = *(const sx8*)(base + (int64_t)qc * tok + 16 * s + 8 * h2);
  // the Q fragments must not share a vmcnt count with the asm DMA below (hipcc cannot count those)
  __builtin_amdgcn_s_waitcnt(0x0F70);
  f32x16 o0 = {}, o1 = {};
  float m = -INFINITY, l = 0.f;
  const int kend = min(T, q0 + A_BQ);
  const int nkt = (kend + A_BK - 1) / A_BK;
  // K and V of this (batch, head): rows of `tok` elements; the resource ends after row T - 1's 64 columns
  const unsigned kv_bytes = (unsigned)(((int64_t)(T - 1) * tok + AD) * 2);
  const u32x4 rK = desc(base + H * AD, kv_bytes), rV = desc(base + 2 * H * AD, kv_bytes);
  // this lane's two pieces (2w, 2w + 1) of a 64 x 64 tile: row r_i, swizzled source chunk ch_i (swz layout)
  int r_[2], c_[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = (w * 2 + i) * 64 + lane, r = p >> 3, k = (r >> 1) & 7;
    r_[i] = r;
    c_[i] = ((p & 7) ^ (((k & 1) << 2) | (k >> 1))) * 8;
  }
  auto issue = [&](int kt, int slot) {  // 4 DMA ops per wave: K pieces 2w, 2w+1, then V pieces
    bf16* sl = sm + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int voff = (int)(((int64_t)min(kt * A_BK + r_[i], T - 1) * tok + c_[i]) * 2);
      dma16(rK, voff, sl + (w * 2 + i) * 512);
    }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int voff = (int)(((int64_t)min(kt * A_BK + r_[i], T - 1) * tok + c_[i]) * 2);
      dma16(rV, voff, sl + A_BK * AD + (w * 2 + i) * 512);
    }
  };
  auto tile = [&](int kt, auto slot_c, auto mask_c) {
    constexpr int slot = decltype(slot_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const bf16* sK = sm + slot * SLOT;
    const bf16* sV = sK + A_BK * AD;
    const int kb = kt * A_BK;
    if (MASK && kb > qw + 31) return;
    f32x16 s0 = {}, s1 = {};
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      s0 = mfma32(row_frag_swz(sK, col, s, h2), qf[s], s0);
      s1 = mfma32(row_frag_swz(sK, 32 + col, s, h2), qf[s], s1);
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
      o0 = mfma32(vt_frag_swz(sV, (s >> 1) * 32, 0, s & 1, lane), pb, o0);
      o1 = mfma32(vt_frag_swz(sV, (s >> 1) * 32, 1, s & 1, lane), pb, o1);
    }
  };
  // step kt: tile kt is visible in slot kt % 3, tile kt + 1 in flight; issue kt + 2 into the slot
  // tile kt - 1 left (every wave passed the barrier behind it), compute kt, then wait for this
  // wave's pieces of kt + 1 (leaving kt + 2's four in flight) and make everyone's visible
  auto step = [&](int kt, auto slot_c, auto mask_c) {
    constexpr int slot = decltype(slot_c)::value;
    const bool more = kt + 2 < nkt;
    if (more) issue(kt + 2, (slot + 2) % 3);
    tile(kt, slot_c, mask_c);
    if (more)
      wait_vm<4>();
    else
      wait_vm<0>();
    barrier();
  };
  issue(0, 0);
  if (nkt > 1) issue(1, 1);
  if (nkt > 1)
    wait_vm<4>();
  else
    wait_vm<0>();
  barrier();
  using I2 = std::integral_constant<int, 2>;
  using Fm = std::false_type;
  using Tm = std::true_type;
  const int kdiag = q0 / A_BK;
  int kt = 0;
  for (; kt + 2 < kdiag; kt += 3) {
    step(kt, I0{}, Fm{});
    step(kt + 1, I1{}, Fm{});
    step(kt + 2, I2{}, Fm{});
  }
  if (kt < kdiag) step(kt++, I0{}, Fm{});  // kt % 3 == 0 here
  if (kt < kdiag) step(kt++, I1{}, Fm{});
  for (; kt < nkt; ++kt) {  // the (at most two) diagonal tiles
    const int sl = kt % 3;
    if (sl == 0)
      step(kt, I0{}, Tm{});
    else if (sl == 1)
      step(kt, I1{}, Tm{});
    else
      step(kt, I2{}, Tm{});
  }
  const float inv = 1.f / l;
  store_acc_tile(o0, o1, inv, out + ((int64_t)b * T + qw) * H * AD + hh * AD, (int64_t)H * AD, T - qw,
                 sm + w * 32 * AD, staged_epi, lane);
  if (q < T && h2 == 0) lse[((int64_t)b * H + hh) * T + q] = m + __log2f(l);
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

// dK / dV with the forward ring's staging ("start with attn_bwd_dkdv"): the Q and
// dO tiles of query tile qt + 2 and that tile's row constants (lse, delta) are issued by inline-asm
// LDS-DMA into a 3-slot ring while tile qt computes; one counted wait (the next tile's 5 ops per wave
// stay in flight) and one raw barrier per tile. The two-buffer kernel above stages through registers
// and drains every load before its ds_writes (vmcnt(0) in 3 of its 7 loop blocks). Row constants
// arrive raw (the -lse and -inf of query rows past T are applied where they are used: every tile that
// holds rows past T runs the masked body, whose mask also drops those rows).
namespace ring {
constexpr int QSLOT = 2 * B_BQ * AD;           // elements: Q tile then dO tile (16 KB)
constexpr int CSLOT = 4 * 256;                 // floats: 1 KB per wave (lse: wave 0, delta: wave 1, 2/3: spare)
constexpr int DK_SLOT_BYTES = QSLOT * 2 + CSLOT * 4;
}  // namespace ring

__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
attn_bwd_dkdv_d64_ring_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const float* __restrict__ lse,
                              const float* __restrict__ delta, bf16* __restrict__ dqkv, float* __restrict__ bpart, int B,
                              int T, int H, float scale, float scale_log2, int staged_epi) {
  using namespace ring;
  __shared__ __attribute__((aligned(16))) char smc[3 * DK_SLOT_BYTES];
  auto sQ_ = [&](int s) { return (bf16*)(smc + s * DK_SLOT_BYTES); };
  auto sD_ = [&](int s) { return (bf16*)(smc + s * DK_SLOT_BYTES) + B_BQ * AD; };
  auto sC_ = [&](int s) { return (float*)(smc + s * DK_SLOT_BYTES + QSLOT * 2); };  // [lse 256 | delta 256 | spare]
  const int tid = threadIdx.x, lane = tid & 63, h2 = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nkb = (T + 127) / 128;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int kbi = lb % nkb;
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
  __builtin_amdgcn_s_waitcnt(0x0F70);  // the K/V fragments: out of the asm DMA's vmcnt accounting
  f32x16 dv0 = {}, dv1 = {}, dk0 = {}, dk1 = {};
  const int qstart = k0 / B_BQ;
  const int nqt = (T + B_BQ - 1) / B_BQ;
  const unsigned q_bytes = (unsigned)(((int64_t)(T - 1) * tok + AD) * 2);
  const unsigned d_bytes = (unsigned)(((int64_t)(T - 1) * otok + AD) * 2);
  const u32x4 rQ = desc(base, q_bytes), rD = desc(dOb, d_bytes);
  const u32x4 rC = desc(w == 1 ? drow : lrow, (unsigned)T * 4u);  // wave 1: delta, the others: lse
  int r_[2], c_[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = (w * 2 + i) * 64 + lane, r = p >> 3, k = (r >> 1) & 7;
    r_[i] = r;
    c_[i] = ((p & 7) ^ (((k & 1) << 2) | (k >> 1))) * 8;
  }
  auto issue = [&](int qt, int slot) {  // 5 DMA ops per wave: Q pieces 2w, 2w+1, dO pieces, row constants
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(rQ, (int)(((int64_t)min(qt * B_BQ + r_[i], T - 1) * tok + c_[i]) * 2), sQ_(slot) + (w * 2 + i) * 512);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(rD, (int)(((int64_t)min(qt * B_BQ + r_[i], T - 1) * otok + c_[i]) * 2), sD_(slot) + (w * 2 + i) * 512);
    // lanes l and l + 16 k read floats qt * 64 + 4 (l & 15) .. + 3 (past T: outside the resource, 0)
    const unsigned m0 = (unsigned)(uintptr_t)(const __attribute__((address_space(3))) float*)(sC_(slot) + w * 256);
    asm volatile("s_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"((qt * B_BQ + 4 * (lane & 15)) * 4),
                 "s"(rC), "{m0}"(m0)
                 : "memory");
  };
  // one 64-query tile; MASK: the diagonal tiles and any tile with query rows past T
  auto tile = [&](int qt, auto slot_c, auto mask_c) {
    constexpr int slot = decltype(slot_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const bf16* sQ = sQ_(slot);
    const bf16* sD = sD_(slot);
    const float* sL = sC_(slot);
    const float* sDel = sC_(slot) + 256;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qb = qt * B_BQ + sub * 32;
      if (MASK && qb + 31 < kw) continue;  // every query before this wave's first key
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(row_frag_swz(sQ, sub * 32 + col, s, h2), kf[s], st);
        dp = mfma32(row_frag_swz(sD, sub * 32 + col, s, h2), vf[s], dp);
      }
      f32x16 pp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *(const f32x4*)(&sL[sub * 32 + 8 * g + 4 * h2]);
        const f32x4 dv = *(const f32x4*)(&sDel[sub * 32 + 8 * g + 4 * h2]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          float p = __builtin_amdgcn_exp2f(fmaf(st[r], scale_log2, -lv[i]));
          if (MASK) {
            const int qq = qb + 8 * g + 4 * h2 + i;
            p = (key > qq || qq >= T) ? 0.f : p;
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
        dv0 = mfma32(vt_frag_swz(sD, sub * 32, 0, s, lane), pb, dv0);
        dv1 = mfma32(vt_frag_swz(sD, sub * 32, 1, s, lane), pb, dv1);
        dk0 = mfma32(vt_frag_swz(sQ, sub * 32, 0, s, lane), sb, dk0);
        dk1 = mfma32(vt_frag_swz(sQ, sub * 32, 1, s, lane), sb, dk1);
      }
    }
  };
  // tile qt sits in slot (qt - qstart) % 3; issue qt + 2 into the slot qt - 1 left, compute qt, wait for
  // this wave's 5 ops of qt + 1 (qt + 2's stay in flight), barrier
  auto step = [&](int qt, auto slot_c, auto mask_c) {
    constexpr int slot = decltype(slot_c)::value;
    const bool more = qt + 2 < nqt;
    if (more) issue(qt + 2, (slot + 2) % 3);
    tile(qt, slot_c, mask_c);
    if (more)
      wait_vm<5>();
    else
      wait_vm<0>();
    barrier();
  };
  using I2 = std::integral_constant<int, 2>;
  using Fm = std::false_type;
  using Tm = std::true_type;
  issue(qstart, 0);
  if (qstart + 1 < nqt) issue(qstart + 1, 1);
  if (qstart + 1 < nqt)
    wait_vm<5>();
  else
    wait_vm<0>();
  barrier();
  // the last tile takes the masked body when it holds query rows past T
  const int nfull = (T % B_BQ) ? nqt - 1 : nqt;  // tiles [.., nfull) have no rows past T
  step(qstart, I0{}, Tm{});  // queries k0 .. k0 + 127 cross the diagonal
  int qt = qstart + 1;
  if (qt < nqt) step(qt++, I1{}, Tm{});
  // slot of qt is (qt - qstart) % 3 = 2 here
  for (; qt + 2 < nfull; qt += 3) {
    step(qt, I2{}, Fm{});
    step(qt + 1, I0{}, Fm{});
    step(qt + 2, I1{}, Fm{});
  }
  for (; qt < nqt; ++qt) {
    const int sl = (qt - qstart) % 3;
    const bool m = qt >= nfull;
    if (sl == 0) {
      if (m) step(qt, I0{}, Tm{}); else step(qt, I0{}, Fm{});
    } else if (sl == 1) {
      if (m) step(qt, I1{}, Tm{}); else step(qt, I1{}, Fm{});
    } else {
      if (m) step(qt, I2{}, Tm{}); else step(qt, I2{}, Fm{});
    }
  }
  bf16* sm0 = (bf16*)smc;
  if (bpart) {  // column sums of this block's dK and dV rows: slots 1 and 2 of a QKV-bias partial row
    float* red = (float*)smc;  // the ring is dead after the loop's last barrier (every DMA retired)
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
  store_acc_tile(dk0, dk1, scale, dk_row0, tok, T - kw, sm0 + w * 32 * AD, staged_epi, lane);
  store_acc_tile(dv0, dv1, 1.f, dk_row0 + H * AD, tok, T - kw, sm0 + 4 * 32 * AD + w * 32 * AD, staged_epi, lane);
}

// dQ with the ring staging of the forward (K / V tiles of key tile kt + 2 in flight while kt computes)
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
attn_bwd_dq_d64_ring_kernel(const bf16* __restrict__ qkv, const bf16* __restrict__ dout, const bf16* __restrict__ out,
                            const float* __restrict__ lse, float* __restrict__ delta, bf16* __restrict__ dqkv,
                            float* __restrict__ bpart, int B, int T, int H, float scale, float scale_log2,
                            int staged_epi) {
  using namespace ring;
  __shared__ __attribute__((aligned(16))) bf16 sm[3 * SLOT];
  const int tid = threadIdx.x, lane = tid & 63, h2 = lane >> 5, col = lane & 31;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = nqt - 1 - (lb % nqt);
  const int bh = lb / nqt;
  const int b = bh / H, hh = bh % H;
  const int64_t tok = 3ll * H * AD;
  const bf16* base = qkv + (int64_t)b * T * tok + hh * AD;
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
  const f32x16 lq16 = splat16(nlq);
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
  __builtin_amdgcn_s_waitcnt(0x0F70);  // every compiler-issued load / store retired before the asm DMA
  const f32x16 dl16 = splat16(-dq_delta);
#pragma unroll
  for (int s = 0; s < 4; ++s) qf[s] = prescale(qf[s], scale_log2);
  f32x16 a0 = {}, a1 = {};
  const int kend = min(T, q0 + A_BQ);
  const int nkt = (kend + A_BK - 1) / A_BK;
  const unsigned kv_bytes = (unsigned)(((int64_t)(T - 1) * tok + AD) * 2);
  const u32x4 rK = desc(base + H * AD, kv_bytes), rV = desc(base + 2 * H * AD, kv_bytes);
  int r_[2], c_[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int p = (w * 2 + i) * 64 + lane, r = p >> 3, k = (r >> 1) & 7;
    r_[i] = r;
    c_[i] = ((p & 7) ^ (((k & 1) << 2) | (k >> 1))) * 8;
  }
  auto issue = [&](int kt, int slot) {
    bf16* sl = sm + slot * SLOT;
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(rK, (int)(((int64_t)min(kt * A_BK + r_[i], T - 1) * tok + c_[i]) * 2), sl + (w * 2 + i) * 512);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      dma16(rV, (int)(((int64_t)min(kt * A_BK + r_[i], T - 1) * tok + c_[i]) * 2), sl + A_BK * AD + (w * 2 + i) * 512);
  };
  auto tile = [&](int kt, auto slot_c, auto mask_c) {
    constexpr int slot = decltype(slot_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const bf16* sK = sm + slot * SLOT;
    const bf16* sV = sK + A_BK * AD;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = kt * A_BK + sub * 32;
      if (MASK && kb > qw + 31) continue;
      f32x16 st = lq16, dp = dl16;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        st = mfma32(row_frag_swz(sK, sub * 32 + col, s, h2), qf[s], st);
        dp = mfma32(row_frag_swz(sV, sub * 32 + col, s, h2), df[s], dp);
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
        a0 = mfma32(vt_frag_swz(sK, sub * 32, 0, s, lane), db, a0);
        a1 = mfma32(vt_frag_swz(sK, sub * 32, 1, s, lane), db, a1);
      }
    }
  };
  auto step = [&](int kt, auto slot_c, auto mask_c) {
    constexpr int slot = decltype(slot_c)::value;
    const bool more = kt + 2 < nkt;
    if (more) issue(kt + 2, (slot + 2) % 3);
    tile(kt, slot_c, mask_c);
    if (more)
      wait_vm<4>();
    else
      wait_vm<0>();
    barrier();
  };
  using I2 = std::integral_constant<int, 2>;
  using Fm = std::false_type;
  using Tm = std::true_type;
  issue(0, 0);
  if (nkt > 1) issue(1, 1);
  if (nkt > 1)
    wait_vm<4>();
  else
    wait_vm<0>();
  barrier();
  const int kdiag = q0 / A_BK;
  int kt = 0;
  for (; kt + 2 < kdiag; kt += 3) {
    step(kt, I0{}, Fm{});
    step(kt + 1, I1{}, Fm{});
    step(kt + 2, I2{}, Fm{});
  }
  if (kt < kdiag) step(kt++, I0{}, Fm{});
  if (kt < kdiag) step(kt++, I1{}, Fm{});
  for (; kt < nkt; ++kt) {
    const int sl = kt % 3;
    if (sl == 0)
      step(kt, I0{}, Tm{});
    else if (sl == 1)
      step(kt, I1{}, Tm{});
    else
      step(kt, I2{}, Tm{});
  }
  store_acc_tile(a0, a1, scale, dqkv + ((int64_t)b * T + qw) * tok + hh * AD, tok, T - qw,  // slot 0 = dQ
                 sm + w * 32 * AD, staged_epi, lane);
  if (bpart) {
    float v[32];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      v[r] = q < T ? a0[r] * scale : 0.f;
      v[16 + r] = q < T ? a1[r] * scale : 0.f;
    }
    const float cs = half_colsum32(v, col);
    float* red = (float*)(sm + SLOT);  // past the dQ images (slot 0 holds them)
    red[w * AD + acc_pair_col(col, h2)] = cs;
    __syncthreads();
    if (tid < AD)
      bpart[((int64_t)b * nqt + qt) * 3 * H * AD + hh * AD + tid] =
          (red[tid] + red[AD + tid]) + (red[2 * AD + tid] + red[3 * AD + tid]);
  }
}

}  // namespace vcx

using namespace vcx;

// Forward default: LDS-DMA staging at 3 waves per SIMD. Measured at the GPT-2 bench shape
// (B=64 H=12 T=1024, one process, interleaved rounds; scripts/attn_variants.py): 0.211 ms, vs
// 0.223 DMA at 2 waves/SIMD, 0.237 register staging at 2 and 0.266 register staging at 3 (spills).
// Backward kernels: 2 waves per SIMD (at 3-4 they spill: dq 0.87-1.25 ms vs 0.64 for the pair);
// dQ with LDS-DMA staging (264 vs 275 us), dK/dV with register staging (381 vs 383 us: the DMA
// build of that kernel hits the 256-VGPR cap and spills).
// Round 6 defaults: the forward and dK/dV on the 3-slot inline-asm LDS-DMA ring (fwd_dma = 2, bwd bit 2): same
// box, interleaved medians (profiles/r6_attention_ring.txt): forward 0.1937 vs 0.2080 ms, backward 0.5571 vs
// 0.5852 ms, outputs bit-identical at T = 1024 / 200 / 202; bench 1063.2 / 1063.0 vs 1053.6 samples/s. The dQ
// kernel on the ring (bit 3) measured even (0.5837 ms) then; built without SLP vectorisation (_build.py FILE_FLAGS)
// it is ahead: backward 0.5278 (both rings, bits 12) vs 0.5337 ms (bits 5), outputs bit-identical
// (gpurun_out/attab, scripts/attn_ring_ab.py) -- now the default.
static int g_fwd_wpe = 3, g_fwd_dma = 2, g_bwd_dma = 12;  // g_bwd_dma bit 0: dQ LDS-DMA, 1: dK/dV LDS-DMA, 2: dK/dV ring, 3: dQ ring
// output tiles (O, dQ, dK, dV): 1 = staged through LDS, whole-row 16-B stores; 0 = per-lane half-row
// stores. Bench shape, same box (profiles/r1_attn_variants.log): backward 0.589 vs 0.614 ms, forward
// within noise (0.201-0.212 vs 0.206-0.208)
static int g_stage_epi = 1;

void vcx_attn_set_variant(int fwd_wpe, int fwd_dma, int bwd_dma, int stage_epi);
// VCX_ATTN="fwd_wpe,fwd_dma,bwd_dma" overrides the defaults once, at the first launch (bench A/B)
static void env_variant() {
  static const bool once = [] {
    const char* e = std::getenv("VCX_ATTN");
    int a = -1, b = -1, c = -1;
    if (e && std::sscanf(e, "%d,%d,%d", &a, &b, &c) == 3) vcx_attn_set_variant(a, b, c, -1);
    return true;
  }();
  (void)once;
}

void vcx_attn_set_variant(int fwd_wpe, int fwd_dma, int bwd_dma, int stage_epi) {
  if (fwd_wpe == 2 || fwd_wpe == 3) g_fwd_wpe = fwd_wpe;
  if (fwd_dma >= 0 && fwd_dma <= 2) g_fwd_dma = fwd_dma;  // 2: the 3-slot ring (attn_fwd_d64_ring_kernel)
  if (bwd_dma >= 0 && bwd_dma <= 15) g_bwd_dma = bwd_dma;  // bit 2: dK/dV on the 3-slot ring, bit 3: dQ on it
  if (stage_epi == 0 || stage_epi == 1) g_stage_epi = stage_epi;
}

int vcx_attn_bias_partials(int B, int T) { return B * ((T + 127) / 128); }

void vcx_attn_bwd_d64(const void* qkv, const void* out, const void* dout, const float* lse, float* delta, void* dqkv,
                      float* bias_part, int B, int T, int H, float scale, hipStream_t s) {
  env_variant();
  // dQ first: it also computes delta = rowsum(dO * O) for the dK/dV kernel
  const int nkb = (T + 127) / 128;
  const int nqt = (T + A_BQ - 1) / A_BQ;
  if (g_bwd_dma & 8)
    hipLaunchKernelGGL(attn_bwd_dq_d64_ring_kernel, dim3(B * H * nqt), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, (const bf16*)out, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale,
                       scale * LOG2E, g_stage_epi);
  else if (g_bwd_dma & 1)
    hipLaunchKernelGGL((attn_bwd_dq_d64_kernel<2, true>), dim3(B * H * nqt), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, (const bf16*)out, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale,
                       scale * LOG2E, g_stage_epi);
  else
    hipLaunchKernelGGL((attn_bwd_dq_d64_kernel<2, false>), dim3(B * H * nqt), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, (const bf16*)out, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale,
                       scale * LOG2E, g_stage_epi);
  if ((g_bwd_dma & 4) && T % 4 == 0)  // the row-constant DMA reads 16-B groups of lse / delta rows
    hipLaunchKernelGGL(attn_bwd_dkdv_d64_ring_kernel, dim3(B * H * nkb), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale, scale * LOG2E,
                       g_stage_epi);
  else if (g_bwd_dma & 2)
    hipLaunchKernelGGL((attn_bwd_dkdv_d64_kernel<2, true>), dim3(B * H * nkb), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale, scale * LOG2E,
                       g_stage_epi);
  else
    hipLaunchKernelGGL((attn_bwd_dkdv_d64_kernel<2, false>), dim3(B * H * nkb), dim3(256), 0, s, (const bf16*)qkv,
                       (const bf16*)dout, lse, delta, (bf16*)dqkv, bias_part, B, T, H, scale, scale * LOG2E,
                       g_stage_epi);
}

void vcx_attn_fwd_d64(const void* qkv, void* out, float* lse, int B, int T, int H, float scale, hipStream_t s) {
  env_variant();
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const dim3 g(B * H * nqt);
#define VCX_FWD(W, D)                                                                                      \
  hipLaunchKernelGGL((attn_fwd_d64_kernel<W, D>), g, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out, lse, B, T, H, \
                     scale * LOG2E, g_stage_epi)
  if (g_fwd_dma == 2) {
    if (g_fwd_wpe == 2)
      hipLaunchKernelGGL((attn_fwd_d64_ring_kernel<2>), g, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out, lse, B, T, H,
                         scale * LOG2E, g_stage_epi);
    else
      hipLaunchKernelGGL((attn_fwd_d64_ring_kernel<3>), g, dim3(256), 0, s, (const bf16*)qkv, (bf16*)out, lse, B, T, H,
                         scale * LOG2E, g_stage_epi);
  } else if (g_fwd_dma) {
    if (g_fwd_wpe == 2) VCX_FWD(2, true); else VCX_FWD(3, true);
  } else {
    if (g_fwd_wpe == 2) VCX_FWD(2, false); else VCX_FWD(3, false);
  }
#undef VCX_FWD
}
