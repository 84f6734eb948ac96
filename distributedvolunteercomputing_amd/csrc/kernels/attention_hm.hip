// Causal flash attention on the head-major grouped-query layout of the Llama family, head dim 64 or
// 128, bf16 in/out, fp32 softmax. Same tile algorithm and MFMA structure as attention.hip (S^T =
// K Q^T with the query on the lane, P^T straight from the accumulator into O^T += V^T P^T, LDS-DMA
// into XOR-swizzled images, deferred rescale), generalised in three ways:
//
//   layout : q [B, Hq, T, D], k / v [B, Hkv, T, D] (what rope_qkv writes); out / dout [B, T, Hq, D]
//            (token-major: the o-projection reads it without a transpose); lse / delta [B, Hq, T]
//            (log2 domain); dq [B, Hq, T, D], dk / dv [B, Hkv, T, D] (what rope_qkv's backward reads)
//   GQA    : query head h reads key/value head h / (Hq / Hkv); the key-parallel dK/dV kernel sums its
//            group's Hq / Hkv query heads inside one workgroup (no atomics, deterministic)
//   D = 128: a tile row is two 64-column halves, each its own swizzled [rows][64] image, so the
//            fragment reads and DMA helpers of attn_common.h apply per half; the O / dQ / dK / dV
//            accumulators are one pair of 32x32 tiles per half. At D = 128 dK and dV run as two
//            launches of the key-parallel kernel (MODE 1 / 2): together their accumulators plus the
//            register-resident K and V fragments exceed the 256-VGPR budget of 2 waves per SIMD.
#include "attn_common.h"
#include "vcx_api.h"

namespace vcx {

constexpr int HM_BQ = 64;  // queries per LDS tile of the key-parallel kernel

template <int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
attn_hm_fwd_kernel(const bf16* __restrict__ qg, const bf16* __restrict__ kg, const bf16* __restrict__ vg,
                   bf16* __restrict__ out, float* __restrict__ lse, int T, int Hq, int Hkv, float scale_log2) {
  constexpr int ND = D / 64;
  __shared__ __attribute__((aligned(16))) bf16 sB0[2 * ND][A_BK * 64];  // [K halves | V halves], swz images
  __shared__ __attribute__((aligned(16))) bf16 sB1[2 * ND][A_BK * 64];
#define sK_(b, h) ((b) ? &sB1[h][0] : &sB0[h][0])
#define sV_(b, h) ((b) ? &sB1[ND + (h)][0] : &sB0[ND + (h)][0])
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h2 = lane >> 5, col = lane & 31;
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = nqt - 1 - (lb % nqt);  // heaviest (last) query tiles first
  const int bh = lb / nqt;              // b * Hq + query head
  const int b = bh / Hq, hh = bh % Hq, hk = hh / (Hq / Hkv);
  const bf16* Qb = qg + (int64_t)bh * T * D;
  const bf16* Kb = kg + ((int64_t)b * Hkv + hk) * T * D;
  const bf16* Vb = vg + ((int64_t)b * Hkv + hk) * T * D;
  const int q0 = qt * A_BQ, qw = q0 + w * 32, q = qw + col, qc = min(q, T - 1);
  sx8 qf[ND][4];
#pragma unroll
  for (int dh = 0; dh < ND; ++dh)
#pragma unroll
    for (int s = 0; s < 4; ++s) qf[dh][s] = *(const sx8*)(Qb + (int64_t)qc * D + dh * 64 + 16 * s + 8 * h2);
  f32x16 o[ND][2] = {};
  float m = -INFINITY, l = 0.f;
  const int kend = min(T, q0 + A_BQ);
  const int nkt = (kend + A_BK - 1) / A_BK;
  auto gload = [&](int kt, int buf) {
#pragma unroll
    for (int dh = 0; dh < ND; ++dh) {
      dma_tile_swz(Kb + dh * 64, D, kt * A_BK, T - 1, sK_(buf, dh), w, lane);
      dma_tile_swz(Vb + dh * 64, D, kt * A_BK, T - 1, sV_(buf, dh), w, lane);
    }
  };
  auto tile = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const int kb = kt * A_BK;
    if (MASK && kb > qw + 31) return;
    f32x16 s0 = {}, s1 = {};
#pragma unroll
    for (int dh = 0; dh < ND; ++dh)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        s0 = mfma32(row_frag_swz(sK_(cur, dh), col, s, h2), qf[dh][s], s0);
        s1 = mfma32(row_frag_swz(sK_(cur, dh), 32 + col, s, h2), qf[dh][s], s1);
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
    if (!__all(mx - m <= 8.f)) {  // deferred rescale, threshold 2^8
      const float mnew = fmaxf(m, mx);
      const float alpha = __builtin_amdgcn_exp2f(m - mnew);
      l *= alpha;
#pragma unroll
      for (int dh = 0; dh < ND; ++dh)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          o[dh][0][r] *= alpha;
          o[dh][1][r] *= alpha;
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
#pragma unroll
      for (int dh = 0; dh < ND; ++dh) {
        o[dh][0] = mfma32(vt_frag_swz(sV_(cur, dh), (s >> 1) * 32, 0, s & 1, lane), pb, o[dh][0]);
        o[dh][1] = mfma32(vt_frag_swz(sV_(cur, dh), (s >> 1) * 32, 1, s & 1, lane), pb, o[dh][1]);
      }
    }
  };
  gload(0, 0);
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);  // retire the Q fragment loads too (see attention.hip)
  const int kdiag = q0 / A_BK;
  auto step = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (kt + 1 < nkt) gload(kt + 1, cur ^ 1);
    tile(kt, cur_c, mask_c);
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
#pragma unroll
  for (int dh = 0; dh < ND; ++dh)  // image of half dh: 4 waves x 32 x 64 in sB0 (dead after the loop)
    store_acc_tile(o[dh][0], o[dh][1], inv, out + ((int64_t)b * T + qw) * Hq * D + hh * D + dh * 64, (int64_t)Hq * D,
                   T - qw, &sB0[0][0] + dh * 4 * 32 * 64 + w * 32 * 64, true, lane);
  if (q < T && h2 == 0) lse[(int64_t)bh * T + q] = m + __log2f(l);
#undef sK_
#undef sV_
}

// dQ (query-parallel) and delta = rowsum(dO * O): the d64 dQ kernel of attention.hip per D-half
template <int D>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(D == 128 ? 1 : 2, D == 128 ? 1 : 2)))
attn_hm_dq_kernel(const bf16* __restrict__ qg, const bf16* __restrict__ kg, const bf16* __restrict__ vg,
                  const bf16* __restrict__ out, const bf16* __restrict__ dout, const float* __restrict__ lse,
                  float* __restrict__ delta, bf16* __restrict__ dq, int T, int Hq, int Hkv, float scale,
                  float scale_log2) {
  constexpr int ND = D / 64;
  __shared__ __attribute__((aligned(16))) bf16 sB0[2 * ND][A_BK * 64];  // [K halves | V halves]
  __shared__ __attribute__((aligned(16))) bf16 sB1[2 * ND][A_BK * 64];
#define sK_(b, h) ((b) ? &sB1[h][0] : &sB0[h][0])
#define sV_(b, h) ((b) ? &sB1[ND + (h)][0] : &sB0[ND + (h)][0])
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h2 = lane >> 5, col = lane & 31;
  const int nqt = (T + A_BQ - 1) / A_BQ;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int qt = nqt - 1 - (lb % nqt);
  const int bh = lb / nqt;
  const int b = bh / Hq, hh = bh % Hq, hk = hh / (Hq / Hkv);
  const bf16* Qb = qg + (int64_t)bh * T * D;
  const bf16* Kb = kg + ((int64_t)b * Hkv + hk) * T * D;
  const bf16* Vb = vg + ((int64_t)b * Hkv + hk) * T * D;
  const int64_t ors = (int64_t)Hq * D;  // token-major row stride of out / dout
  const int q0 = qt * A_BQ, qw = q0 + w * 32, q = qw + col, qc = min(q, T - 1);
  const bf16* dOr = dout + ((int64_t)b * T + qc) * ors + hh * D;
  const bf16* Or = out + ((int64_t)b * T + qc) * ors + hh * D;
  sx8 qf[ND][4], df[ND][4];
  float acc = 0.f;
#pragma unroll
  for (int dh = 0; dh < ND; ++dh)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      qf[dh][s] = *(const sx8*)(Qb + (int64_t)qc * D + dh * 64 + 16 * s + 8 * h2);
      df[dh][s] = *(const sx8*)(dOr + dh * 64 + 16 * s + 8 * h2);
      const sx8 ov = *(const sx8*)(Or + dh * 64 + 16 * s + 8 * h2);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const short ob = ov[j], db = df[dh][s][j];
        acc = fmaf((float)*(const bf16*)&ob, (float)*(const bf16*)&db, acc);
      }
    }
  const float dq_delta = xhalf_sum(acc);
  if (h2 == 0 && q < T) delta[(int64_t)bh * T + q] = dq_delta;
  const float nlq = -lse[(int64_t)bh * T + qc];
  f32x16 a[ND][2] = {};
  const int kend = min(T, q0 + A_BQ);
  const int nkt = (kend + A_BK - 1) / A_BK;
  auto gload = [&](int kt, int buf) {
#pragma unroll
    for (int dh = 0; dh < ND; ++dh) {
      dma_tile_swz(Kb + dh * 64, D, kt * A_BK, T - 1, sK_(buf, dh), w, lane);
      dma_tile_swz(Vb + dh * 64, D, kt * A_BK, T - 1, sV_(buf, dh), w, lane);
    }
  };
  auto tile = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int kb = kt * A_BK + sub * 32;
      if (MASK && kb > qw + 31) continue;
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int dh = 0; dh < ND; ++dh) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(row_frag_swz(sK_(cur, dh), sub * 32 + col, s, h2), qf[dh][s], st);
          dp = mfma32(row_frag_swz(sV_(cur, dh), sub * 32 + col, s, h2), df[dh][s], dp);
        }
        if constexpr (ND > 1) __builtin_amdgcn_sched_barrier(0);  // see the dK/dV kernel
      }
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float p = __builtin_amdgcn_exp2f(fmaf(st[r], scale_log2, nlq));
        if (MASK) {
          const int key = kb + (r & 3) + 8 * (r >> 2) + 4 * h2;
          p = key > q ? 0.f : p;
        }
        st[r] = p * (dp[r] - dq_delta);  // dS^T
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        sx8 db;
#pragma unroll
        for (int j = 0; j < 8; ++j) db[j] = bf16_bits(st[8 * s + j]);
#pragma unroll
        for (int dh = 0; dh < ND; ++dh) {
          if constexpr (ND > 1) __builtin_amdgcn_sched_barrier(0);
          a[dh][0] = mfma32(vt_frag_swz(sK_(cur, dh), sub * 32, 0, s, lane), db, a[dh][0]);
          a[dh][1] = mfma32(vt_frag_swz(sK_(cur, dh), sub * 32, 1, s, lane), db, a[dh][1]);
        }
      }
    }
  };
  gload(0, 0);
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);
  const int kdiag = q0 / A_BK;
  auto step = [&](int kt, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (kt + 1 < nkt) gload(kt + 1, cur ^ 1);
    tile(kt, cur_c, mask_c);
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
#pragma unroll
  for (int dh = 0; dh < ND; ++dh)
    store_acc_tile(a[dh][0], a[dh][1], scale, dq + ((int64_t)bh * T + qw) * D + dh * 64, D, T - qw,
                   &sB0[0][0] + dh * 4 * 32 * 64 + w * 32 * 64, true, lane);
#undef sK_
#undef sV_
}

// dK and/or dV (key-parallel, key on the lane) for one key/value head: the workgroup's 128 keys
// stay in registers while it streams the Q / dO tiles of every query head of the group in turn
// (one flattened tile sequence, so the double-buffered prefetch runs across head boundaries).
// MODE 0: dK and dV; 1: dK only; 2: dV only.
// waves per SIMD of the key-parallel kernel: D = 64 both gradients at 2; D = 128 dK (and dK + dV)
// needs the 512-register budget of 1 wave per SIMD, dV alone fits 3
constexpr int hm_dkv_wpe(int D, int MODE) { return D == 64 ? 2 : (MODE == 2 ? 3 : 1); }

template <int D, int MODE>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(hm_dkv_wpe(D, MODE), hm_dkv_wpe(D, MODE))))
attn_hm_dkv_kernel(const bf16* __restrict__ qg, const bf16* __restrict__ kg, const bf16* __restrict__ vg,
                   const bf16* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ delta,
                   bf16* __restrict__ dk, bf16* __restrict__ dv, int T, int Hq, int Hkv, float scale,
                   float scale_log2) {
  constexpr int ND = D / 64;
  constexpr bool DK = MODE != 2, DV = MODE != 1;
  __shared__ __attribute__((aligned(16))) bf16 sQD0[2 * ND][HM_BQ * 64];  // [Q halves | dO halves]
  __shared__ __attribute__((aligned(16))) bf16 sQD1[2 * ND][HM_BQ * 64];
#define sQ_(b, h) ((b) ? &sQD1[h][0] : &sQD0[h][0])
#define sD_(b, h) ((b) ? &sQD1[ND + (h)][0] : &sQD0[ND + (h)][0])
  __shared__ __attribute__((aligned(16))) float sL[2][HM_BQ];
  __shared__ __attribute__((aligned(16))) float sDel[2][HM_BQ];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h2 = lane >> 5, col = lane & 31;
  const int nkb = (T + 127) / 128;
  const int lb = xcd_remap(blockIdx.x, gridDim.x);
  const int kbi = lb % nkb;
  const int bhk = lb / nkb;  // b * Hkv + key/value head
  const int b = bhk / Hkv, hk = bhk % Hkv, rep = Hq / Hkv;
  const bf16* Kb = kg + (int64_t)bhk * T * D;
  const bf16* Vb = vg + (int64_t)bhk * T * D;
  const int64_t ors = (int64_t)Hq * D;
  const int k0 = kbi * 128, kw = k0 + w * 32, key = kw + col, kc = min(key, T - 1);
  sx8 kf[ND][4], vf[ND][4];
#pragma unroll
  for (int dh = 0; dh < ND; ++dh)
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      kf[dh][s] = *(const sx8*)(Kb + (int64_t)kc * D + dh * 64 + 16 * s + 8 * h2);
      if constexpr (DK) vf[dh][s] = *(const sx8*)(Vb + (int64_t)kc * D + dh * 64 + 16 * s + 8 * h2);
    }
  f32x16 gk[ND][2] = {}, gv[ND][2] = {};
  const int qstart = k0 / HM_BQ;  // first query tile that can see these keys
  const int nqt = (T + HM_BQ - 1) / HM_BQ;
  const int nq = nqt - qstart;    // query tiles per head
  const int total = rep * nq;
  float rl = 0.f, rdl = 0.f;
  auto gload = [&](int idx, int buf) {
    const int hq = hk * rep + idx / nq, qt = qstart + idx % nq;
    const bf16* Qb = qg + ((int64_t)b * Hq + hq) * T * D;
    const bf16* dOb = dout + (int64_t)b * T * ors + hq * D;
#pragma unroll
    for (int dh = 0; dh < ND; ++dh) {
      dma_tile_swz(Qb + dh * 64, D, qt * HM_BQ, T - 1, sQ_(buf, dh), w, lane);
      dma_tile_swz(dOb + dh * 64, ors, qt * HM_BQ, T - 1, sD_(buf, dh), w, lane);
    }
    if (tid < HM_BQ) {  // -lse (P = exp2(S c + nl)); -inf for rows past T: their P is 0
      const int qq = qt * HM_BQ + tid;
      const int64_t rb = ((int64_t)b * Hq + hq) * T;
      rl = qq < T ? -lse[rb + qq] : -INFINITY;
      rdl = delta[rb + min(qq, T - 1)];
    }
  };
  auto sstore = [&](int buf) {
    if (tid < HM_BQ) {
      sL[buf][tid] = rl;
      sDel[buf][tid] = rdl;
    }
  };
  auto tile = [&](int idx, auto cur_c, auto mask_c) {
    constexpr int cur = decltype(cur_c)::value;
    constexpr bool MASK = decltype(mask_c)::value;
    const int qt = qstart + idx % nq;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int qb = qt * HM_BQ + sub * 32;
      if (MASK && qb + 31 < kw) continue;  // every query before this wave's first key
      f32x16 st = {}, dp = {};
#pragma unroll
      for (int dh = 0; dh < ND; ++dh) {
#pragma unroll
        for (int s = 0; s < 4; ++s) {
          st = mfma32(row_frag_swz(sQ_(cur, dh), sub * 32 + col, s, h2), kf[dh][s], st);
          if constexpr (DK) dp = mfma32(row_frag_swz(sD_(cur, dh), sub * 32 + col, s, h2), vf[dh][s], dp);
        }
        // keep the next half's fragment reads behind this half's MFMAs: at D = 128 hoisting all of
        // them runs the kernel out of registers
        if constexpr (ND > 1) __builtin_amdgcn_sched_barrier(0);
      }
      f32x16 pp;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const f32x4 lv = *(const f32x4*)(&sL[cur][sub * 32 + 8 * g + 4 * h2]);
        const f32x4 dl = *(const f32x4*)(&sDel[cur][sub * 32 + 8 * g + 4 * h2]);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int r = 4 * g + i;
          float p = __builtin_amdgcn_exp2f(fmaf(st[r], scale_log2, lv[i]));
          if (MASK) {
            const int qq = qb + 8 * g + 4 * h2 + i;
            p = key > qq ? 0.f : p;
          }
          pp[r] = p;
          if constexpr (DK) st[r] = p * (dp[r] - dl[i]);  // dS
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
#pragma unroll
        for (int dh = 0; dh < ND; ++dh) {
          if constexpr (ND > 1) __builtin_amdgcn_sched_barrier(0);
          if constexpr (DV) {
            gv[dh][0] = mfma32(vt_frag_swz(sD_(cur, dh), sub * 32, 0, s, lane), pb, gv[dh][0]);
            gv[dh][1] = mfma32(vt_frag_swz(sD_(cur, dh), sub * 32, 1, s, lane), pb, gv[dh][1]);
          }
          if constexpr (DK) {
            gk[dh][0] = mfma32(vt_frag_swz(sQ_(cur, dh), sub * 32, 0, s, lane), sb, gk[dh][0]);
            gk[dh][1] = mfma32(vt_frag_swz(sQ_(cur, dh), sub * 32, 1, s, lane), sb, gk[dh][1]);
          }
        }
      }
    }
  };
  gload(0, 0);
  sstore(0);
  __syncthreads();
  __builtin_amdgcn_s_waitcnt(0x0F70);
  // the first two query tiles of every head cross this block's diagonal (128 keys = 2 tiles)
  auto step = [&](int idx, auto cur_c) {
    constexpr int cur = decltype(cur_c)::value;
    if (idx + 1 < total) gload(idx + 1, cur ^ 1);
    if (idx % nq < 2)
      tile(idx, cur_c, std::true_type{});
    else
      tile(idx, cur_c, std::false_type{});
    if (idx + 1 < total) sstore(cur ^ 1);
    __syncthreads();
  };
  int idx = 0;
  for (; idx + 1 < total; idx += 2) {
    step(idx, I0{});
    step(idx + 1, I1{});
  }
  if (idx < total) step(idx, I0{});
  const int64_t orow = (int64_t)bhk * T + kw;
#pragma unroll
  for (int dh = 0; dh < ND; ++dh) {
    if constexpr (DK)
      store_acc_tile(gk[dh][0], gk[dh][1], scale, dk + orow * D + dh * 64, D, T - kw,
                     &sQD0[0][0] + dh * 4 * 32 * 64 + w * 32 * 64, true, lane);
    if constexpr (DV)
      store_acc_tile(gv[dh][0], gv[dh][1], 1.f, dv + orow * D + dh * 64, D, T - kw,
                     &sQD1[0][0] + dh * 4 * 32 * 64 + w * 32 * 64, true, lane);
  }
#undef sQ_
#undef sD_
}

}  // namespace vcx

using namespace vcx;

void vcx_attn_hm_fwd(const void* q, const void* k, const void* v, void* out, float* lse, int B, int T, int Hq, int Hkv,
                     int D, float scale, hipStream_t s) {
  const dim3 g(B * Hq * ((T + A_BQ - 1) / A_BQ));
  if (D == 128)
    hipLaunchKernelGGL(attn_hm_fwd_kernel<128>, g, dim3(256), 0, s, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       (bf16*)out, lse, T, Hq, Hkv, scale * LOG2E);
  else
    hipLaunchKernelGGL(attn_hm_fwd_kernel<64>, g, dim3(256), 0, s, (const bf16*)q, (const bf16*)k, (const bf16*)v,
                       (bf16*)out, lse, T, Hq, Hkv, scale * LOG2E);
}

static int g_hm_dkv_split = 0;  // D = 128: dK and dV as two launches (1) or one 1-wave/SIMD launch (0)
void vcx_attn_hm_set_variant(int dkv_split) {
  if (dkv_split == 0 || dkv_split == 1) g_hm_dkv_split = dkv_split;
}

void vcx_attn_hm_bwd(const void* q, const void* k, const void* v, const void* out, const void* dout, const float* lse,
                     float* delta, void* dq, void* dk, void* dv, int B, int T, int Hq, int Hkv, int D, float scale,
                     hipStream_t s) {
  const dim3 gq(B * Hq * ((T + A_BQ - 1) / A_BQ)), gk(B * Hkv * ((T + 127) / 128));
  const float sl = scale * LOG2E;
#define VCX_HM_ARGS_Q (const bf16*)q, (const bf16*)k, (const bf16*)v
  if (D == 128) {
    hipLaunchKernelGGL(attn_hm_dq_kernel<128>, gq, dim3(256), 0, s, VCX_HM_ARGS_Q, (const bf16*)out, (const bf16*)dout,
                       lse, delta, (bf16*)dq, T, Hq, Hkv, scale, sl);
    if (g_hm_dkv_split) {
      hipLaunchKernelGGL((attn_hm_dkv_kernel<128, 1>), gk, dim3(256), 0, s, VCX_HM_ARGS_Q, (const bf16*)dout, lse,
                         delta, (bf16*)dk, (bf16*)dv, T, Hq, Hkv, scale, sl);
      hipLaunchKernelGGL((attn_hm_dkv_kernel<128, 2>), gk, dim3(256), 0, s, VCX_HM_ARGS_Q, (const bf16*)dout, lse,
                         delta, (bf16*)dk, (bf16*)dv, T, Hq, Hkv, scale, sl);
    } else {
      hipLaunchKernelGGL((attn_hm_dkv_kernel<128, 0>), gk, dim3(256), 0, s, VCX_HM_ARGS_Q, (const bf16*)dout, lse,
                         delta, (bf16*)dk, (bf16*)dv, T, Hq, Hkv, scale, sl);
    }
  } else {
    hipLaunchKernelGGL(attn_hm_dq_kernel<64>, gq, dim3(256), 0, s, VCX_HM_ARGS_Q, (const bf16*)out, (const bf16*)dout,
                       lse, delta, (bf16*)dq, T, Hq, Hkv, scale, sl);
    hipLaunchKernelGGL((attn_hm_dkv_kernel<64, 0>), gk, dim3(256), 0, s, VCX_HM_ARGS_Q, (const bf16*)dout, lse, delta,
                       (bf16*)dk, (bf16*)dv, T, Hq, Hkv, scale, sl);
  }
#undef VCX_HM_ARGS_Q
}
