// Gradient / pseudo-gradient compression kernels (gfx950): exact top-k with error feedback
// and PowerSGD rank-r with error feedback. No reference analog (BASELINE.json
// configs 3 and 5).
//
// Top-k: the k-th largest |g + e| is found EXACTLY by a 3-pass radix select on the IEEE bit
// pattern of |x| (monotonic for non-negative floats): 12 + 12 + 7 bits. Pass 1 (fused with the
// error-feedback accumulation) is a per-block LDS histogram of the top 12 bits; passes 2 and 3
// read x again and histogram ONLY the elements inside the chosen bin (a few per mille); a
// 1-block scan after each pass narrows the prefix. All state stays on the device (no host sync; graph-capturable). Selection then
// compacts the winners: elements above the threshold fill the output from the front, ties with
// it from the back, both claimed with ONE 64-bit atomic per 16k elements.
//
// HBM traffic per element: 10 B (accumulate: g 2 + e 4 read, e 4 written) + 2 x 4 B (passes 2,
// 3) + 4 B (select) = 22 B.
//
// PowerSGD (Vogels et al. 2019): M <- g + e; P = M Q; allreduce(P); P = orth(P);
// Q = M^T P; allreduce(Q); out = P Q^T; e = M - out. For rank r <= 8 the two products are
// HBM-bound (2r FLOP per 4-B element), so they are single-pass streaming kernels with the
// small Q/P operands served from L2; all matrices of a model are processed by ONE launch per
// stage through a device-side descriptor table (grouped kernels).
#include "vcx_common.h"

namespace vcx {

// =====================================================================================
// top-k
// =====================================================================================
// state layout (int32): [0] prefix bits, [1] remaining k (after the last pass: the tie budget),
//                       [3] threshold bits, [6..7] 64-bit output claim counter (above | ties << 32)
constexpr int TK_BINS = 4096;

__device__ __forceinline__ uint32_t absbits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

// acc = g + e (written to e, fp32), histogram pass 1 of |acc| (bits 30..19 -> 12 bits).
// 8 elements per lane per step (one 16-B g load for bf16, two 16-B e loads/stores).
template <typename GT>
__device__ __forceinline__ void load8(const GT* __restrict__ g, int64_t i, float (&a)[8]) {
  if constexpr (sizeof(GT) == 2) {
    const bf16x8 v = *(const bf16x8*)(g + i);
#pragma unroll
    for (int j = 0; j < 8; ++j) a[j] = (float)v[j];
  } else {
    const f32x4 u = *(const f32x4*)(g + i), w = *(const f32x4*)(g + i + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] = u[j];
      a[j + 4] = w[j];
    }
  }
}

template <typename GT>
__global__ void __launch_bounds__(256) topk_accum_hist_kernel(const GT* __restrict__ g, float* __restrict__ e,
                                                               int64_t n, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[TK_BINS];
  for (int i = threadIdx.x; i < TK_BINS; i += 256) h[i] = 0;
  __syncthreads();
  const bool vec = ((((uintptr_t)g) | ((uintptr_t)e)) & 15) == 0;
  const int64_t n8 = vec ? n / 8 : 0;
  for (int64_t v = blockIdx.x * 256ll + threadIdx.x; v < n8; v += (int64_t)gridDim.x * 256) {
    float a[8];
    load8(g, v * 8, a);
    f32x4 e0 = *(const f32x4*)(e + v * 8), e1 = *(const f32x4*)(e + v * 8 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      e0[j] += a[j];
      e1[j] += a[j + 4];
    }
    *(f32x4*)(e + v * 8) = e0;
    *(f32x4*)(e + v * 8 + 4) = e1;
    // per-lane LDS atomics: same-bin lanes serialise inside the LDS, which costs far less than a
    // ballot-leader loop over the ~30 distinct bins of a wave's gradient values
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      atomicAdd(&h[absbits(e0[j]) >> 19], 1u);
      atomicAdd(&h[absbits(e1[j]) >> 19], 1u);
    }
  }
  for (int64_t i = n8 * 8 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float a = (float)g[i] + e[i];
    e[i] = a;
    atomicAdd(&h[absbits(a) >> 19], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TK_BINS; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// passes 2 and 3: histogram of the next bit field (`nbits` bits at `shift`) over the elements
// whose higher bits equal the current prefix. Only those few per mille take part: a per-lane
// LDS atomic each, one global atomic per nonzero bin per block at the end.
__global__ void __launch_bounds__(256) topk_hist_kernel(const float* __restrict__ x, int64_t n,
                                                         const int* __restrict__ st, int shift_hi, int shift,
                                                         int nbits, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[TK_BINS];
  const int nb = 1 << nbits;
  for (int i = threadIdx.x; i < nb; i += 256) h[i] = 0;
  __syncthreads();
  const uint32_t prefix = (uint32_t)st[0];
  const bool vec = (((uintptr_t)x) & 15) == 0;
  const int64_t n8 = vec ? n / 8 : 0;
  for (int64_t v = blockIdx.x * 256ll + threadIdx.x; v < n8; v += (int64_t)gridDim.x * 256) {
    const f32x4 a = *(const f32x4*)(x + v * 8), b = *(const f32x4*)(x + v * 8 + 4);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const uint32_t u = absbits(j < 4 ? a[j] : b[j - 4]);
      if ((u >> shift_hi) == prefix) atomicAdd(&h[(u >> shift) & (nb - 1)], 1u);
    }
  }
  for (int64_t i = n8 * 8 + blockIdx.x * 256ll + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const uint32_t u = absbits(x[i]);
    if ((u >> shift_hi) == prefix) atomicAdd(&h[(u >> shift) & (nb - 1)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// one block of T threads: find the bin (from the top) where the cumulative count reaches the
// remaining k; extend the prefix by it; update remaining k. Thread t owns the t-th chunk of
// nb / T bins counted from the top; a block scan of the chunk sums finds the one chunk where the
// count crosses, and only that thread walks its bins. `hist` is re-zeroed by the launcher.
// (A 19-bit second pass into a global histogram was tried: bf16 gradients put every hit of the
// 12-bit bin on 8 of its 2^19 bins and the global atomics serialised — 3.7 ms.)
template <int T>
__global__ void __launch_bounds__(T) topk_scan_kernel(const uint32_t* __restrict__ hist, int nbits,
                                                       int* __restrict__ st, int last) {
  __shared__ uint32_t ws[T / 64];
  const int nb = 1 << nbits;
  const int rem = st[1];
  const uint32_t pre = (uint32_t)st[0];
  const int t = threadIdx.x, lane = t & 63, wid = t >> 6;
  const int C = (nb + T - 1) / T;
  const int hi = max(0, nb - t * C), lo = max(0, hi - C);
  uint32_t sum = 0;
  for (int b = lo; b < hi; ++b) sum += hist[b];
  uint32_t incl = sum;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) ws[wid] = incl;
  __syncthreads();
  uint32_t before = 0, total = 0;
#pragma unroll
  for (int w = 0; w < T / 64; ++w) {
    before += w < wid ? ws[w] : 0u;
    total += ws[w];
  }
  const uint32_t excl = before + incl - sum;
  const uint32_t need = (uint32_t)rem;
  int bin = -1;
  uint32_t cum = excl;
  if (hi > lo && excl < need && excl + sum >= need) {
    for (int b = hi - 1; b >= lo; --b) {
      if (cum + hist[b] >= need) {
        bin = b;
        break;
      }
      cum += hist[b];
    }
  } else if (t == T - 1 && total < need) {  // fewer candidates than rem: keep them all (bin 0)
    bin = 0;
    cum = total;
  }
  if (bin >= 0) {
    st[0] = (int)((pre << nbits) | (uint32_t)bin);
    st[1] = rem - (int)cum;  // how many elements equal to the final prefix we still need
    if (last) st[3] = st[0];  // full 31-bit pattern of the k-th largest magnitude
  }
}

// compact: |x| > thr always selected (filling the output from the front); |x| == thr selected
// while the tie budget st[1] lasts (filling it from the back). Selected entries are removed from
// the error buffer (error feedback keeps the rest).
// A block step covers TOPK_SUB sub-steps of 256 x TOPK_EPT elements (TOPK_EPT / 4 coalesced
// f32x4 loads per lane each); per sub-step a lane keeps only two 32-bit masks (above / tie, parked
// in LDS), the values die as soon as the masks are built and the few winners are re-read when
// written out (holding the values across the claim needed 226 VGPRs: 2 waves/SIMD). The step claims its
// output slots with ONE 64-bit atomic on st[6..7] (low word: above count, high word: ties) —
// one per 32k elements: the claims on that single address serialise in L2 (16k claims: 0.37 ms,
// 32k: 0.51 ms for 268M elements). Bf16 gradients put tens of thousands of elements exactly on the
// threshold value; the old per-wave tie atomic on one address took 2.9 ms.
constexpr int TOPK_EPT = 32;  // values per lane per sub-step (fits the 32-bit masks)
constexpr int TOPK_SUB = 4;   // sub-steps per claim: packed 16-bit block counts stay <= 32768

template <typename VT>
__global__ void __launch_bounds__(256) topk_select_kernel(float* __restrict__ x, int64_t n, int* __restrict__ st,
                                                           int k, int32_t* __restrict__ idx_out,
                                                           VT* __restrict__ val_out) {
  __shared__ uint32_t wsum[4];
  __shared__ unsigned long long bbase;
  __shared__ uint32_t sgm[TOPK_SUB][256], stm[TOPK_SUB][256];  // per-lane masks of the sub-steps
  const uint32_t thr = (uint32_t)st[3];
  const int tie_budget = st[1];
  unsigned long long* claim = (unsigned long long*)(st + 6);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool vec = (((uintptr_t)x) & 15) == 0;
  constexpr int64_t SUBSTEP = 256ll * TOPK_EPT, STEP = SUBSTEP * TOPK_SUB;
  for (int64_t base = blockIdx.x * STEP; base < n; base += (int64_t)gridDim.x * STEP) {
    // element j of sub-step u for this lane: base + u * SUBSTEP + (j / 4) * 1024 + 4 * threadIdx.x + (j % 4)
    uint32_t mine = 0;
#pragma unroll 1
    for (int u = 0; u < TOPK_SUB; ++u) {  // not unrolled: one sub-step of values live at a time
      const int64_t sb = base + u * SUBSTEP;
      float v[TOPK_EPT];
#pragma unroll
      for (int c = 0; c < TOPK_EPT / 4; ++c) {
        const int64_t i0 = sb + (int64_t)c * 1024 + 4 * threadIdx.x;
        if (vec && i0 + 3 < n) {
          const f32x4 t = *(const f32x4*)(x + i0);
#pragma unroll
          for (int j = 0; j < 4; ++j) v[c * 4 + j] = t[j];
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j) v[c * 4 + j] = (i0 + j < n) ? x[i0 + j] : 0.f;
        }
      }
      uint32_t g = 0, t = 0;
#pragma unroll
      for (int j = 0; j < TOPK_EPT; ++j) {
        const uint32_t b = absbits(v[j]);
        g |= (uint32_t)(b > thr) << j;
        t |= (uint32_t)(b == thr && b != 0u) << j;  // zero padding never ties
      }
      sgm[u][threadIdx.x] = g;
      stm[u][threadIdx.x] = t;
      mine += (uint32_t)__popc(g) | ((uint32_t)__popc(t) << 16);  // packed (above | ties << 16)
    }
    uint32_t incl = mine;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
      const uint32_t tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
      bbase = tot ? atomicAdd(claim, (unsigned long long)(tot & 0xffffu) | ((unsigned long long)(tot >> 16) << 32))
                  : 0ull;
    }
    __syncthreads();
    uint32_t excl = incl - mine;
    for (int w = 0; w < wid; ++w) excl += wsum[w];
    const unsigned long long bb = bbase;
    int pos = (int)(uint32_t)bb + (int)(excl & 0xffffu);
    int tie = (int)(uint32_t)(bb >> 32) + (int)(excl >> 16);
#pragma unroll 1
    for (int u = 0; u < TOPK_SUB; ++u) {
      const uint32_t gmu = sgm[u][threadIdx.x], tmu = stm[u][threadIdx.x];
      for (uint32_t m = gmu | tmu; m; m &= m - 1) {  // ascending (u, j): the order of the counts
        const int j = __builtin_ctz(m);
        const bool isg = (gmu >> j) & 1u;
        const int slot = isg ? pos : k - 1 - tie;
        const bool take = isg ? pos < k : tie < tie_budget;
        pos += isg;
        tie += !isg;
        if (take) {
          const int64_t i = base + u * SUBSTEP + (int64_t)(j >> 2) * 1024 + 4 * threadIdx.x + (j & 3);
          const float val = x[i];
          const VT sent = (VT)val;
          idx_out[slot] = (int32_t)i;
          val_out[slot] = sent;
          x[i] = val - (float)sent;  // the wire-dtype rounding residual stays in error feedback
        }
      }
    }
    __syncthreads();  // wsum / bbase are rewritten by the next step
  }
}

// dense[idx[j]] += scale * val[j]  (fp32 accumulation of gathered sparse contributions).
// Indices outside [0, n) are dropped in the kernel (no host-side max/min sync per round).
// zero values are skipped: slots the selection left unfilled (fewer than k nonzero candidates)
// hold idx 0 / val 0, and thousands of no-op atomics on dense[0] serialised the kernel (3.2 ms)
template <typename VT>
__global__ void __launch_bounds__(256) scatter_add_kernel(const int32_t* __restrict__ idx, const VT* __restrict__ val,
                                                           int64_t m, float scale, float* __restrict__ dense,
                                                           int64_t n) {
  for (int64_t j = blockIdx.x * 256ll + threadIdx.x; j < m; j += (int64_t)gridDim.x * 256) {
    const float v = (float)val[j];
    const uint32_t i = (uint32_t)idx[j];
    if (v != 0.f && i < (uint32_t)n) atomicAdd(&dense[i], scale * v);
  }
}

// the all-gathered wire format of P peers: per peer L int32 words = k indices, then k values
// (VT) packed into the following words
template <typename VT>
__global__ void __launch_bounds__(256) scatter_add_packed_kernel(const int32_t* __restrict__ wire, int P, int k,
                                                                  int64_t L, float scale, float* __restrict__ dense,
                                                                  int64_t n) {
  const int64_t m = (int64_t)P * k;
  for (int64_t j = blockIdx.x * 256ll + threadIdx.x; j < m; j += (int64_t)gridDim.x * 256) {
    const int64_t p = j / k, r = j - p * k;
    const int32_t* w = wire + p * L;
    const float v = (float)((const VT*)(w + k))[r];
    const uint32_t i = (uint32_t)w[r];
    if (v != 0.f && i < (uint32_t)n) atomicAdd(&dense[i], scale * v);
  }
}

// =====================================================================================
// PowerSGD (grouped over matrices)
// =====================================================================================
struct MatDesc {
  int64_t off;   // element offset of M in the flat fp32 buffer
  int64_t poff;  // element offset of P [rows, R]
  int64_t qoff;  // element offset of Q [cols, R]
  int rows, cols;
  int blk0;      // first block of this matrix in the current launch's block numbering
  int pad;
};

__device__ __forceinline__ int find_mat(const MatDesc* __restrict__ d, int nmat, int b, int stage) {
  // blk0 for stage s is stored in descriptor table s (caller passes the table for the stage)
  int lo = 0, hi = nmat - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (d[mid].blk0 <= b) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// R consecutive fp32 values (a row of P or Q) — 16-B loads when R is a multiple of 4 (P / Q
// offsets are multiples of R, so those rows are 16-B aligned)
template <int R>
__device__ __forceinline__ void load_rv(const float* __restrict__ p, float (&v)[R]) {
  if constexpr (R % 4 == 0) {
#pragma unroll
    for (int i = 0; i < R; i += 4) {
      const f32x4 t = *(const f32x4*)(p + i);
      v[i] = t[0];
      v[i + 1] = t[1];
      v[i + 2] = t[2];
      v[i + 3] = t[3];
    }
  } else {
#pragma unroll
    for (int i = 0; i < R; ++i) v[i] = p[i];
  }
}

// matrices whose flat offset and row length are multiples of 4 take the 16-B paths below
__device__ __forceinline__ bool psgd_vec(const MatDesc& md) { return ((md.off | (int64_t)md.cols) & 3) == 0; }

// psgd_mq / psgd_reconstruct: each wave owns PSGD_ROWS consecutive rows of a matrix (16 per block)
// and sweeps their columns, so every Q fragment it loads serves PSGD_ROWS rows (one row per wave
// read R floats of Q per element of M: 4x the M traffic at R = 4, through L2).
constexpr int PSGD_ROWS = 4;

// P[row, :] = M[row, :] . Q with the error-feedback accumulation M += G fused into this first pass
// over M (G == nullptr: no accumulation). On the 16-B path each lane takes 4 consecutive columns
// per step (f32x4 M load/store, 8-B G load per row).
// LAZY: the previous round's reconstruct left M = e + P Q^T (it only wrote the output), so this
// pass first subtracts P_prev Q^T from each element (P_prev = this wave's P rows as they stand, Q =
// the warm-start Q, i.e. exactly the pair the previous reconstruct used): e = M - P_prev Q^T + G.
// That moves the error-feedback update out of reconstruct, whose pass then never touches M
// (2 x 4 B per element less HBM traffic per round), at R extra FMAs per element here.
template <int R, bool LAZY>
__global__ void __launch_bounds__(256) psgd_mq_kernel(const MatDesc* __restrict__ d, int nmat, float* __restrict__ M,
                                                       const bf16* __restrict__ G, const float* __restrict__ Q,
                                                       float* __restrict__ P) {
  const int mi = find_mat(d, nmat, blockIdx.x, 0);
  const MatDesc md = d[mi];
  const int rw = ((blockIdx.x - md.blk0) * 4 + (threadIdx.x >> 6)) * PSGD_ROWS;
  const int lane = threadIdx.x & 63;
  if (rw >= md.rows) return;
  const int nr = min(PSGD_ROWS, md.rows - rw);  // wave-uniform
  const int64_t rb = md.off + (int64_t)rw * md.cols;
  const float* q = Q + md.qoff;
  float acc[PSGD_ROWS][R];
  float pold[PSGD_ROWS][R];
#pragma unroll
  for (int i = 0; i < PSGD_ROWS; ++i) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[i][r] = pold[i][r] = 0.f;
    if (LAZY && i < nr) load_rv<R>(P + md.poff + (int64_t)(rw + i) * R, pold[i]);
  }
  if (psgd_vec(md)) {
    for (int c = 4 * lane; c < md.cols; c += 256) {
      float qv[4][R];
#pragma unroll
      for (int j = 0; j < 4; ++j) load_rv<R>(q + (int64_t)(c + j) * R, qv[j]);
#pragma unroll
      for (int i = 0; i < PSGD_ROWS; ++i) {
        if (i < nr) {
          const int64_t e = rb + (int64_t)i * md.cols + c;
          f32x4 mv = *(const f32x4*)(M + e);
          if (LAZY) {
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              float s = 0.f;
#pragma unroll
              for (int r = 0; r < R; ++r) s = fmaf(pold[i][r], qv[j][r], s);
              mv[j] -= s;
            }
          }
          if (G) {
            const bf16x4 gv = *(const bf16x4*)(G + e);
#pragma unroll
            for (int j = 0; j < 4; ++j) mv[j] += (float)gv[j];
          }
          if (LAZY || G) *(f32x4*)(M + e) = mv;
#pragma unroll
          for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < R; ++r) acc[i][r] = fmaf(mv[j], qv[j][r], acc[i][r]);
        }
      }
    }
  } else {
    for (int c = lane; c < md.cols; c += 64) {
      float qv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) qv[r] = q[(int64_t)c * R + r];
#pragma unroll
      for (int i = 0; i < PSGD_ROWS; ++i) {
        if (i < nr) {
          const int64_t e = rb + (int64_t)i * md.cols + c;
          float mv = M[e];
          if (LAZY) {
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < R; ++r) s = fmaf(pold[i][r], qv[r], s);
            mv -= s;
          }
          if (G) mv += (float)G[e];
          if (LAZY || G) M[e] = mv;
#pragma unroll
          for (int r = 0; r < R; ++r) acc[i][r] = fmaf(mv, qv[r], acc[i][r]);
        }
      }
    }
  }
#pragma unroll
  for (int i = 0; i < PSGD_ROWS; ++i) {
    if (i < nr) {
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float s = wave_sum(acc[i][r]);
        if (lane == 0) P[md.poff + (int64_t)(rw + i) * R + r] = s;
      }
    }
  }
}

// Q[c, :] += sum over a 256-row slab of M[row, c] * P[row, :]   (Q zeroed beforehand)
// block = (matrix, row slab of 256, column chunk of 256): each wave sweeps 64 rows of the slab for
// 4 consecutive columns per lane (one f32x4 M load per row on the 16-B path, P's slab broadcast
// from LDS); the 4 waves' partials are summed in LDS and added to Q with coalesced atomics
// (consecutive lanes -> consecutive Q words, R / 256 atomics per element of M).
constexpr int PSGD_MTP_ROWS = 256, PSGD_MTP_COLS = 256;

template <int R>
__global__ void __launch_bounds__(256) psgd_mtp_kernel(const MatDesc* __restrict__ d, int nmat,
                                                        const float* __restrict__ M, const float* __restrict__ P,
                                                        float* __restrict__ Q) {
  const int mi = find_mat(d, nmat, blockIdx.x, 1);
  const MatDesc md = d[mi];
  const int local = blockIdx.x - md.blk0;
  const int nck = (md.cols + PSGD_MTP_COLS - 1) / PSGD_MTP_COLS;
  const int slab = local / nck, ck = local % nck;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int r0 = slab * PSGD_MTP_ROWS;
  __shared__ float sp[PSGD_MTP_ROWS][R];
  __shared__ float red[4][PSGD_MTP_COLS * R];
  for (int i = threadIdx.x; i < PSGD_MTP_ROWS * R; i += 256) {
    const int rr = r0 + i / R;
    sp[i / R][i % R] = rr < md.rows ? P[md.poff + (int64_t)rr * R + (i % R)] : 0.f;
  }
  __syncthreads();
  const int c = ck * PSGD_MTP_COLS + 4 * lane;
  const int wr0 = r0 + 64 * w, wr1 = min(wr0 + 64, md.rows);
  float acc[4][R];
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < R; ++r) acc[j][r] = 0.f;
  if (c < md.cols) {
    const float* mb = M + md.off + c;
    if (psgd_vec(md)) {  // cols % 4 == 0: all 4 columns are in range
#pragma unroll 8
      for (int row = wr0; row < wr1; ++row) {
        const f32x4 mv = *(const f32x4*)(mb + (int64_t)row * md.cols);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int r = 0; r < R; ++r) acc[j][r] = fmaf(mv[j], sp[row - r0][r], acc[j][r]);
      }
    } else {
      for (int row = wr0; row < wr1; ++row) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const float mv = c + j < md.cols ? mb[(int64_t)row * md.cols + j] : 0.f;
#pragma unroll
          for (int r = 0; r < R; ++r) acc[j][r] = fmaf(mv, sp[row - r0][r], acc[j][r]);
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j)
#pragma unroll
    for (int r = 0; r < R; ++r) red[w][(4 * lane + j) * R + r] = acc[j][r];
  __syncthreads();
  float* qc = Q + md.qoff + (int64_t)ck * PSGD_MTP_COLS * R;
  for (int i = threadIdx.x; i < PSGD_MTP_COLS * R; i += 256)
    if (ck * PSGD_MTP_COLS + i / R < md.cols) atomicAdd(qc + i, red[0][i] + red[1][i] + red[2][i] + red[3][i]);
}

// modified Gram-Schmidt on the R columns of each P (one block per matrix)
// orth(P) for every matrix at once, as CholeskyQR2 in coefficient space: the R x R Gram
// G = P^T P of each matrix is reduced over row slabs by many blocks (one pass over P); every
// block then derives the upper-triangular T with (P T)^T (P T) = I by modified Gram-Schmidt on
// G (R^3 flops, redundantly per thread) and rewrites its rows P <- P T, accumulating the Gram of
// the result for the second, re-orthogonalising round. Three launches, three streaming passes
// over P with every CU busy, instead of the old one-block-per-matrix serial Gram-Schmidt
// (R(R+1) dependent block reductions per matrix: 1.73 ms for Llama-3-8B's 224 matrices).
// For R <= 8 the Gram is R(R+1)/2 dot products per row — a VALU reduction; MFMA tiles would
// be >90% padding.
constexpr int ORTH_RPT = 8;  // rows per thread -> 2048-row slabs per block

template <int R>
__device__ __forceinline__ void orth_coeffs(const float* __restrict__ Gs, float (&t)[R][R]) {
  // Gs: upper triangle of the symmetric Gram, Gs[a*R+b] for a <= b
  auto G = [&](int a, int b) { return a <= b ? Gs[a * R + b] : Gs[b * R + a]; };
#pragma unroll
  for (int i = 0; i < R; ++i) {
#pragma unroll
    for (int k = 0; k < R; ++k) t[i][k] = (k == i) ? 1.f : 0.f;
#pragma unroll
    for (int j = 0; j < i; ++j) {  // c = q_j^T v_i = t_j^T G t_i
      float c = 0.f;
#pragma unroll
      for (int a = 0; a <= j; ++a)
#pragma unroll
        for (int b = 0; b <= i; ++b) c = fmaf(t[j][a] * G(a, b), t[i][b], c);
#pragma unroll
      for (int k = 0; k <= j; ++k) t[i][k] -= c * t[j][k];
    }
    float nrm = 0.f;
#pragma unroll
    for (int a = 0; a <= i; ++a)
#pragma unroll
      for (int b = 0; b <= i; ++b) nrm = fmaf(t[i][a] * G(a, b), t[i][b], nrm);
    const float inv = nrm > 1e-30f ? rsqrtf(nrm) : 0.f;  // a null column stays zero
#pragma unroll
    for (int k = 0; k <= i; ++k) t[i][k] *= inv;
  }
}

// mode 0: Gram of P into Gout. mode 1: P <- P T(Gin), Gram of the result into Gout. mode 2:
// P <- P T(Gin) only.
template <int R, int MODE>
__global__ void __launch_bounds__(256) psgd_orth_pass_kernel(const MatDesc* __restrict__ d, int nmat,
                                                              float* __restrict__ P, const float* __restrict__ Gin,
                                                              float* __restrict__ Gout) {
  constexpr int NG = R * (R + 1) / 2;
  __shared__ float part[4][NG];
  const int mi = find_mat(d, nmat, blockIdx.x, 0);
  const MatDesc md = d[mi];
  float t[R][R];
  if constexpr (MODE != 0) orth_coeffs<R>(Gin + (int64_t)mi * R * R, t);
  float acc[NG];
#pragma unroll
  for (int q = 0; q < NG; ++q) acc[q] = 0.f;
  const int row0 = (blockIdx.x - md.blk0) * 256 * ORTH_RPT;
  float* p = P + md.poff;
#pragma unroll 2
  for (int rr = 0; rr < ORTH_RPT; ++rr) {
    const int row = row0 + rr * 256 + threadIdx.x;
    if (row < md.rows) {
      float v[R];
      load_rv<R>(p + (int64_t)row * R, v);
      if constexpr (MODE != 0) {
        float w[R];
#pragma unroll
        for (int i = 0; i < R; ++i) {
          float a = 0.f;
#pragma unroll
          for (int k = 0; k <= i; ++k) a = fmaf(v[k], t[i][k], a);
          w[i] = a;
        }
#pragma unroll
        for (int i = 0; i < R; ++i) {
          v[i] = w[i];
          p[(int64_t)row * R + i] = w[i];
        }
      }
      if constexpr (MODE != 2) {
        int q = 0;
#pragma unroll
        for (int a = 0; a < R; ++a)
#pragma unroll
          for (int b = a; b < R; ++b) {
            acc[q] = fmaf(v[a], v[b], acc[q]);
            ++q;
          }
      }
    }
  }
  if constexpr (MODE != 2) {
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
    for (int q = 0; q < NG; ++q) {
      const float r = wave_sum(acc[q]);
      if (lane == 0) part[wid][q] = r;
    }
    __syncthreads();
    if (threadIdx.x < NG) {
      const int q = threadIdx.x;
      int a = 0, rem = q;
      while (rem >= R - a) {  // q -> (a, b) of the upper triangle, row-major
        rem -= R - a;
        ++a;
      }
      const int b = a + rem;
      atomicAdd(&Gout[(int64_t)mi * R * R + a * R + b], part[0][q] + part[1][q] + part[2][q] + part[3][q]);
    }
  }
}

// out = P Q^T (bf16, into the flat output buffer at md.off), e = M - P Q^T (in place on M; with
// UPDATE_M false M is left alone and the next psgd_mq<LAZY> applies the subtraction).
// Same row ownership as psgd_mq (PSGD_ROWS rows per wave, P rows held in registers, each Q
// fragment used for all of them); 16-B M load/store and 8-B out store per row on the vector path.
template <int R, bool UPDATE_M>
__global__ void __launch_bounds__(256) psgd_reconstruct_kernel(const MatDesc* __restrict__ d, int nmat,
                                                                float* __restrict__ M, const float* __restrict__ P,
                                                                const float* __restrict__ Q, bf16* __restrict__ out) {
  const int mi = find_mat(d, nmat, blockIdx.x, 2);
  const MatDesc md = d[mi];
  const int rw = ((blockIdx.x - md.blk0) * 4 + (threadIdx.x >> 6)) * PSGD_ROWS;
  const int lane = threadIdx.x & 63;
  if (rw >= md.rows) return;
  const int nr = min(PSGD_ROWS, md.rows - rw);
  const int64_t rb = md.off + (int64_t)rw * md.cols;
  const float* q = Q + md.qoff;
  float pv[PSGD_ROWS][R];
#pragma unroll
  for (int i = 0; i < PSGD_ROWS; ++i) {
    if (i < nr) {
      load_rv<R>(P + md.poff + (int64_t)(rw + i) * R, pv[i]);
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) pv[i][r] = 0.f;
    }
  }
  if (psgd_vec(md)) {
    for (int c = 4 * lane; c < md.cols; c += 256) {
      float qv[4][R];
#pragma unroll
      for (int j = 0; j < 4; ++j) load_rv<R>(q + (int64_t)(c + j) * R, qv[j]);
#pragma unroll
      for (int i = 0; i < PSGD_ROWS; ++i) {
        if (i < nr) {
          f32x4 v;
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            float s = 0.f;
#pragma unroll
            for (int r = 0; r < R; ++r) s = fmaf(pv[i][r], qv[j][r], s);
            v[j] = s;
          }
          const int64_t e = rb + (int64_t)i * md.cols + c;
          if (UPDATE_M) {
            f32x4 mv = *(const f32x4*)(M + e);
            mv -= v;
            *(f32x4*)(M + e) = mv;
          }
          const bf16x4 ov = {(bf16)v[0], (bf16)v[1], (bf16)v[2], (bf16)v[3]};
          *(bf16x4*)(out + e) = ov;
        }
      }
    }
  } else {
    for (int c = lane; c < md.cols; c += 64) {
      float qv[R];
#pragma unroll
      for (int r = 0; r < R; ++r) qv[r] = q[(int64_t)c * R + r];
#pragma unroll
      for (int i = 0; i < PSGD_ROWS; ++i) {
        if (i < nr) {
          float v = 0.f;
#pragma unroll
          for (int r = 0; r < R; ++r) v = fmaf(pv[i][r], qv[r], v);
          const int64_t e = rb + (int64_t)i * md.cols + c;
          if (UPDATE_M) M[e] -= v;
          out[e] = (bf16)v;
        }
      }
    }
  }
}

// e = e + g  (fp32 += bf16) over a flat range; used before PowerSGD
__global__ void __launch_bounds__(256) ef_accum_kernel(const bf16* __restrict__ g, float* __restrict__ e, int64_t n8) {
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n8; i += (int64_t)gridDim.x * 256) {
    bf16x8 gv = *(const bf16x8*)(g + i * 8);
    f32x4 a = *(const f32x4*)(e + i * 8), b = *(const f32x4*)(e + i * 8 + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      a[j] += (float)gv[j];
      b[j] += (float)gv[j + 4];
    }
    *(f32x4*)(e + i * 8) = a;
    *(f32x4*)(e + i * 8 + 4) = b;
  }
}

}  // namespace vcx

// ====================================================================================== launchers
using namespace vcx;

void vcx_topk_ef(const void* g, int g_is_bf16, float* e, int64_t n, int k, int* st, uint32_t* hist,
                 int32_t* idx_out, void* val_out, int val_is_bf16, hipStream_t s) {
  // st = {0, k, 0, 0, 0, 0, 0, 0} (set by the caller); hist: TK_BINS zeroed words, left zeroed
  const int grid = stream_grid(n / 8 + 1, 256, 2048);
  const size_t hb = TK_BINS * sizeof(uint32_t);
  if (g_is_bf16)
    hipLaunchKernelGGL(topk_accum_hist_kernel<bf16>, dim3(grid), dim3(256), 0, s, (const bf16*)g, e, n, hist);
  else
    hipLaunchKernelGGL(topk_accum_hist_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)g, e, n, hist);
  hipLaunchKernelGGL(topk_scan_kernel<256>, dim3(1), dim3(256), 0, s, hist, 12, st, 0);
  hipMemsetAsync(hist, 0, hb, s);
  hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(256), 0, s, e, n, st, 19, 7, 12, hist);
  hipLaunchKernelGGL(topk_scan_kernel<256>, dim3(1), dim3(256), 0, s, hist, 12, st, 0);
  hipMemsetAsync(hist, 0, hb, s);
  hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(256), 0, s, e, n, st, 7, 0, 7, hist);
  hipLaunchKernelGGL(topk_scan_kernel<256>, dim3(1), dim3(256), 0, s, hist, 7, st, 1);
  hipMemsetAsync(hist, 0, hb, s);
  const int sgrid = stream_grid((n + TOPK_EPT * TOPK_SUB - 1) / (TOPK_EPT * TOPK_SUB), 256, 2048);
  if (val_is_bf16)
    hipLaunchKernelGGL(topk_select_kernel<bf16>, dim3(sgrid), dim3(256), 0, s, e, n, st, k, idx_out, (bf16*)val_out);
  else
    hipLaunchKernelGGL(topk_select_kernel<float>, dim3(sgrid), dim3(256), 0, s, e, n, st, k, idx_out,
                       (float*)val_out);
}

int vcx_topk_hist_words() { return TK_BINS; }

void vcx_scatter_add(const int32_t* idx, const void* val, int val_is_bf16, int64_t m, float scale, float* dense,
                     int64_t n, hipStream_t s) {
  const int grid = stream_grid(m, 256, 1024);
  if (val_is_bf16)
    hipLaunchKernelGGL(scatter_add_kernel<bf16>, dim3(grid), dim3(256), 0, s, idx, (const bf16*)val, m, scale, dense,
                       n);
  else
    hipLaunchKernelGGL(scatter_add_kernel<float>, dim3(grid), dim3(256), 0, s, idx, (const float*)val, m, scale,
                       dense, n);
}

void vcx_scatter_add_packed(const int32_t* wire, int P, int k, int64_t L, int val_is_bf16, float scale, float* dense,
                            int64_t n, hipStream_t s) {
  const int grid = stream_grid((int64_t)P * k, 256, 1024);
  if (val_is_bf16)
    hipLaunchKernelGGL(scatter_add_packed_kernel<bf16>, dim3(grid), dim3(256), 0, s, wire, P, k, L, scale, dense, n);
  else
    hipLaunchKernelGGL(scatter_add_packed_kernel<float>, dim3(grid), dim3(256), 0, s, wire, P, k, L, scale, dense, n);
}

#define PSGD_R_DISPATCH(RV, ...)                              \
  switch (RV) {                                               \
    case 1: { constexpr int R = 1; __VA_ARGS__; } break;      \
    case 2: { constexpr int R = 2; __VA_ARGS__; } break;      \
    case 4: { constexpr int R = 4; __VA_ARGS__; } break;      \
    default: { constexpr int R = 8; __VA_ARGS__; } break;     \
  }

void vcx_psgd_mq(const void* desc, int nmat, int nblocks, float* M, const void* G, const float* Q, float* P, int rank,
                 int lazy, hipStream_t s) {
  if (lazy) {
    PSGD_R_DISPATCH(rank, hipLaunchKernelGGL((psgd_mq_kernel<R, true>), dim3(nblocks), dim3(256), 0, s,
                                             (const MatDesc*)desc, nmat, M, (const bf16*)G, Q, P));
  } else {
    PSGD_R_DISPATCH(rank, hipLaunchKernelGGL((psgd_mq_kernel<R, false>), dim3(nblocks), dim3(256), 0, s,
                                             (const MatDesc*)desc, nmat, M, (const bf16*)G, Q, P));
  }
}

void vcx_psgd_mtp(const void* desc, int nmat, int nblocks, const float* M, const float* P, float* Q, int rank,
                  hipStream_t s) {
  PSGD_R_DISPATCH(rank, hipLaunchKernelGGL(psgd_mtp_kernel<R>, dim3(nblocks), dim3(256), 0, s, (const MatDesc*)desc,
                                           nmat, M, P, Q));
}

void vcx_psgd_orth(const void* desc, int nmat, int nblocks, float* P, float* G, int rank, hipStream_t s) {
  // G: 2 * nmat * rank^2 floats of scratch (zeroed here)
  const int64_t gm = (int64_t)nmat * rank * rank;
  hipMemsetAsync(G, 0, 2 * gm * sizeof(float), s);
  PSGD_R_DISPATCH(rank, {
    const MatDesc* d = (const MatDesc*)desc;
    hipLaunchKernelGGL((psgd_orth_pass_kernel<R, 0>), dim3(nblocks), dim3(256), 0, s, d, nmat, P, G, G);
    hipLaunchKernelGGL((psgd_orth_pass_kernel<R, 1>), dim3(nblocks), dim3(256), 0, s, d, nmat, P, G, G + gm);
    hipLaunchKernelGGL((psgd_orth_pass_kernel<R, 2>), dim3(nblocks), dim3(256), 0, s, d, nmat, P, G + gm, G);
  });
}

int vcx_psgd_orth_rows() { return 256 * ORTH_RPT; }

void vcx_psgd_reconstruct(const void* desc, int nmat, int nblocks, float* M, const float* P, const float* Q,
                          void* out, int rank, int update_m, hipStream_t s) {
  if (update_m) {
    PSGD_R_DISPATCH(rank, hipLaunchKernelGGL((psgd_reconstruct_kernel<R, true>), dim3(nblocks), dim3(256), 0, s,
                                             (const MatDesc*)desc, nmat, M, P, Q, (bf16*)out));
  } else {
    PSGD_R_DISPATCH(rank, hipLaunchKernelGGL((psgd_reconstruct_kernel<R, false>), dim3(nblocks), dim3(256), 0, s,
                                             (const MatDesc*)desc, nmat, M, P, Q, (bf16*)out));
  }
}

void vcx_ef_accum(const void* g, float* e, int64_t n, hipStream_t s) {
  hipLaunchKernelGGL(ef_accum_kernel, dim3(stream_grid(n / 8, 256)), dim3(256), 0, s, (const bf16*)g, e, n / 8);
}

int vcx_psgd_desc_size() { return (int)sizeof(MatDesc); }
int vcx_psgd_rows_per_block() { return 4 * PSGD_ROWS; }
int vcx_psgd_mtp_rows() { return PSGD_MTP_ROWS; }
int vcx_psgd_mtp_cols() { return PSGD_MTP_COLS; }
