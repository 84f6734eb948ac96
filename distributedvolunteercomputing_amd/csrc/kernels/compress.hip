// Gradient / pseudo-gradient compression kernels (gfx950): exact top-k with error feedback
// and PowerSGD rank-r with error feedback. No reference analog (BASELINE.json
// configs 3 and 5).
//
// Top-k: the k-th largest |g + e| is found EXACTLY by a 3-pass radix select on the IEEE bit
// pattern of |x| (monotonic for non-negative floats): 12 + 12 + 7 bits, each pass a per-block
// LDS histogram merged with one global atomic per bin, then a 1-block scan that narrows the
// prefix. All state stays on the device (no host sync; graph-capturable). Selection then
// compacts the winners with a per-wave ballot prefix + one atomic per wave.
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
// state layout (int32): [0] prefix bits, [1] remaining k, [2] selected count, [3] threshold bits,
//                       [4] n_greater (elements strictly above threshold)
constexpr int TK_BINS = 4096;

__device__ __forceinline__ uint32_t absbits(float v) { return __float_as_uint(v) & 0x7fffffffu; }

// Wave-aggregated LDS histogram increment: each distinct bin present in the wave costs ONE
// atomic (leader + ballot popcount). Used by the refinement passes, where only the few lanes
// whose value matches the current prefix take part; the first pass, where every lane does,
// uses plain per-lane LDS atomics (cheaper than this loop over ~30 distinct bins).
__device__ __forceinline__ void wave_hist_add(uint32_t* h, int bin, bool valid) {
  unsigned long long todo = __ballot(valid);
  const int lane = threadIdx.x & 63;
  while (todo) {
    const int leader = __ffsll((long long)todo) - 1;
    const int lb = __shfl(bin, leader, 64);
    const unsigned long long same = __ballot(valid && bin == lb) & todo;
    if (lane == leader) atomicAdd(&h[lb], (uint32_t)__popcll(same));
    todo &= ~same;
  }
}

// acc = g + e (written to e, fp32), histogram pass 0 of |acc| (bits 30..19 -> 12 bits)
template <typename GT>
__global__ void __launch_bounds__(256) topk_accum_hist_kernel(const GT* __restrict__ g, float* __restrict__ e,
                                                               int64_t n, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[TK_BINS];
  for (int i = threadIdx.x; i < TK_BINS; i += 256) h[i] = 0;
  __syncthreads();
  // the loop bound is wave-uniform (whole-block strides) so every lane joins the ballots
  for (int64_t base = blockIdx.x * 256ll; base < n; base += (int64_t)gridDim.x * 256) {
    const int64_t i = base + threadIdx.x;
    int bin = 0;
    if (i < n) {
      float a = (float)g[i] + e[i];
      e[i] = a;
      bin = (int)(absbits(a) >> 19);
      // per-lane LDS atomic: same-bin lanes serialise inside the LDS, which costs far less than
      // the wave_hist_add leader loop over the ~30 distinct bins of a wave's gradient values
      // (776 us vs 6.0 ms for 268M elements)
      atomicAdd(&h[bin], 1u);
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < TK_BINS; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// histogram of the next bit field for elements whose higher bits equal the current prefix
__global__ void __launch_bounds__(256) topk_hist_kernel(const float* __restrict__ x, int64_t n,
                                                         const int* __restrict__ st, int shift_hi, int shift,
                                                         int nbits, uint32_t* __restrict__ hist) {
  __shared__ uint32_t h[TK_BINS];
  const int nb = 1 << nbits;
  for (int i = threadIdx.x; i < nb; i += 256) h[i] = 0;
  __syncthreads();
  const uint32_t prefix = (uint32_t)st[0];
  for (int64_t base = blockIdx.x * 256ll; base < n; base += (int64_t)gridDim.x * 256) {
    const int64_t i = base + threadIdx.x;
    bool hit = false;
    int bin = 0;
    if (i < n) {
      const uint32_t b = absbits(x[i]);
      hit = (b >> shift_hi) == prefix;
      bin = (int)((b >> shift) & (nb - 1));
    }
    wave_hist_add(h, bin, hit);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nb; i += 256)
    if (h[i]) atomicAdd(&hist[i], h[i]);
}

// one block: walk the histogram from the top bin down until the cumulative count reaches
// the remaining k; extend the prefix by that bin; update remaining k; zero the histogram.
__global__ void __launch_bounds__(256) topk_scan_kernel(uint32_t* __restrict__ hist, int nbits, int* __restrict__ st,
                                                         int last) {
  __shared__ uint32_t h[TK_BINS];
  const int nb = 1 << nbits;
  for (int i = threadIdx.x; i < nb; i += 256) {
    h[i] = hist[i];
    hist[i] = 0;
  }
  const int rem = st[1];
  const uint32_t pre = (uint32_t)st[0];
  // thread t owns the t-th chunk of C bins counted from the top; a block scan of the chunk sums
  // finds the one chunk where the cumulative count from the top reaches rem, and only that
  // thread walks its C bins (a single-thread walk over 4096 bins took ~210 us per pass)
  __shared__ uint32_t ps[256];
  const int t = threadIdx.x;
  const int C = (nb + 255) / 256;
  const int hi = max(0, nb - t * C), lo = max(0, hi - C);
  __syncthreads();
  uint32_t sum = 0;
  for (int b = lo; b < hi; ++b) sum += h[b];
  ps[t] = sum;
  __syncthreads();
  for (int o = 1; o < 256; o <<= 1) {
    const uint32_t v = t >= o ? ps[t - o] : 0u;
    __syncthreads();
    ps[t] += v;
    __syncthreads();
  }
  const uint32_t excl = ps[t] - sum;
  const uint32_t need = (uint32_t)rem;
  int bin = -1;
  uint32_t cum = excl;
  if (hi > lo && excl < need && excl + sum >= need) {
    for (int b = hi - 1; b >= lo; --b) {
      if (cum + h[b] >= need) {
        bin = b;
        break;
      }
      cum += h[b];
    }
  } else if (t == 255 && ps[255] < need) {  // fewer candidates than rem: keep the lowest bin
    bin = 0;
    cum = ps[255];
  }
  if (bin >= 0) {
    st[0] = (int)((pre << nbits) | (uint32_t)bin);
    st[1] = rem - (int)cum;  // how many elements equal to the final prefix we still need
    if (last) {
      st[3] = st[0];  // full 31-bit pattern of the k-th largest magnitude
      st[2] = 0;
    }
  }
}

// compact: |x| > thr always selected; |x| == thr selected while the tie budget lasts.
// Selected entries are removed from the error buffer (error feedback keeps the rest).
// Each block step covers 256 x TOPK_EPT elements (TOPK_EPT / 4 coalesced f32x4 loads per lane);
// the output slots are claimed with ONE global atomic per block step (wave scan of the per-lane
// counts + LDS across the 4 waves) instead of one per wave: at 1% density about half of all
// 64-element waves hold a selected entry, and those per-wave atomics on the single counter
// serialised the kernel (25 ms for 268M elements; 3.4 ms at 16 elements per lane, one atomic
// per 4096 elements).
constexpr int TOPK_EPT = 64;

template <typename VT>
__global__ void __launch_bounds__(256) topk_select_kernel(float* __restrict__ x, int64_t n, int* __restrict__ st,
                                                           int k, int32_t* __restrict__ idx_out,
                                                           VT* __restrict__ val_out) {
  __shared__ int wsum[4];
  __shared__ int bbase;
  const uint32_t thr = (uint32_t)st[3];
  int* ties = st + 1;
  int* count = st + 2;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const bool vec = (((uintptr_t)x) & 15) == 0;
  constexpr int64_t STEP = 256ll * TOPK_EPT;
  for (int64_t base = blockIdx.x * STEP; base < n; base += (int64_t)gridDim.x * STEP) {
    // element j of this lane: base + (j / 4) * 1024 + 4 * threadIdx.x + (j % 4)
    float v[TOPK_EPT];
#pragma unroll
    for (int c = 0; c < TOPK_EPT / 4; ++c) {
      const int64_t i0 = base + (int64_t)c * 1024 + 4 * threadIdx.x;
      if (vec && i0 + 3 < n) {
        const f32x4 t = *(const f32x4*)(x + i0);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[c * 4 + j] = t[j];
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[c * 4 + j] = (i0 + j < n) ? x[i0 + j] : 0.f;
      }
    }
    uint64_t selm = 0;
#pragma unroll
    for (int j = 0; j < TOPK_EPT; ++j) {
      const uint32_t b = absbits(v[j]);
      bool sel = b > thr;
      // ties with the threshold draw from the tie budget, one atomic per wave (ranked by lane);
      // zero padding never ties (b != 0)
      const bool tie = !sel && b == thr && b != 0u;
      const uint64_t tm = __ballot(tie);
      if (tm) {
        int left = 0;
        if (lane == 0) left = atomicSub(ties, __popcll(tm));
        left = __shfl(left, 0, 64);
        if (tie) sel = __popcll(tm & ((1ull << lane) - 1ull)) < left;
      }
      selm |= (uint64_t)sel << j;
    }
    const int cnt = __popcll(selm);
    int incl = cnt;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int t = __shfl_up(incl, o, 64);
      if (lane >= o) incl += t;
    }
    if (lane == 63) wsum[wid] = incl;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int tot = wsum[0] + wsum[1] + wsum[2] + wsum[3];
      bbase = tot ? atomicAdd(count, tot) : 0;
    }
    __syncthreads();
    int pos = bbase + incl - cnt;
    for (int w = 0; w < wid; ++w) pos += wsum[w];
#pragma unroll
    for (int j = 0; j < TOPK_EPT; ++j) {
      if ((selm >> j) & 1ull) {
        const int64_t i = base + (int64_t)(j >> 2) * 1024 + 4 * threadIdx.x + (j & 3);
        if (pos < k) {
          const VT sent = (VT)v[j];
          idx_out[pos] = (int32_t)i;
          val_out[pos] = sent;
          x[i] = v[j] - (float)sent;  // the wire-dtype rounding residual stays in error feedback
        }
        ++pos;
      }
    }
    __syncthreads();  // wsum / bbase are rewritten by the next step
  }
}

// dense[idx[j]] += scale * val[j]  (fp32 accumulation of gathered sparse contributions)
template <typename VT>
__global__ void __launch_bounds__(256) scatter_add_kernel(const int32_t* __restrict__ idx, const VT* __restrict__ val,
                                                           int64_t m, float scale, float* __restrict__ dense) {
  // zero values are skipped: slots the selection left unfilled (fewer than k nonzero candidates)
  // hold idx 0 / val 0, and thousands of no-op atomics on dense[0] serialised the kernel (3.2 ms)
  for (int64_t j = blockIdx.x * 256ll + threadIdx.x; j < m; j += (int64_t)gridDim.x * 256) {
    const float v = (float)val[j];
    if (v != 0.f) atomicAdd(&dense[idx[j]], scale * v);
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
template <int R>
__global__ void __launch_bounds__(256) psgd_orth_kernel(const MatDesc* __restrict__ d, float* __restrict__ P) {
  __shared__ float scratch[4];
  const MatDesc md = d[blockIdx.x];
  float* p = P + md.poff;
  for (int i = 0; i < R; ++i) {
    for (int j = 0; j < i; ++j) {
      float s = 0.f;
      for (int row = threadIdx.x; row < md.rows; row += 256) s = fmaf(p[(int64_t)row * R + i], p[(int64_t)row * R + j], s);
      s = block_sum<256>(s, scratch);
      for (int row = threadIdx.x; row < md.rows; row += 256) p[(int64_t)row * R + i] -= s * p[(int64_t)row * R + j];
      __syncthreads();
    }
    float s = 0.f;
    for (int row = threadIdx.x; row < md.rows; row += 256) {
      const float v = p[(int64_t)row * R + i];
      s = fmaf(v, v, s);
    }
    s = block_sum<256>(s, scratch);
    const float inv = 1.f / (sqrtf(s) + 1e-8f);
    for (int row = threadIdx.x; row < md.rows; row += 256) p[(int64_t)row * R + i] *= inv;
    __syncthreads();
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
  const int grid = stream_grid(n, 256, 1024);
  // st[0] = prefix 0, st[1] = k (set by the caller with a memset-free init kernel below)
  if (g_is_bf16)
    hipLaunchKernelGGL(topk_accum_hist_kernel<bf16>, dim3(grid), dim3(256), 0, s, (const bf16*)g, e, n, hist);
  else
    hipLaunchKernelGGL(topk_accum_hist_kernel<float>, dim3(grid), dim3(256), 0, s, (const float*)g, e, n, hist);
  hipLaunchKernelGGL(topk_scan_kernel, dim3(1), dim3(256), 0, s, hist, 12, st, 0);
  hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(256), 0, s, e, n, st, 19, 7, 12, hist);
  hipLaunchKernelGGL(topk_scan_kernel, dim3(1), dim3(256), 0, s, hist, 12, st, 0);
  hipLaunchKernelGGL(topk_hist_kernel, dim3(grid), dim3(256), 0, s, e, n, st, 7, 0, 7, hist);
  hipLaunchKernelGGL(topk_scan_kernel, dim3(1), dim3(256), 0, s, hist, 7, st, 1);
  const int sgrid = stream_grid((n + TOPK_EPT - 1) / TOPK_EPT, 256, 1024);
  if (val_is_bf16)
    hipLaunchKernelGGL(topk_select_kernel<bf16>, dim3(sgrid), dim3(256), 0, s, e, n, st, k, idx_out, (bf16*)val_out);
  else
    hipLaunchKernelGGL(topk_select_kernel<float>, dim3(sgrid), dim3(256), 0, s, e, n, st, k, idx_out,
                       (float*)val_out);
}

void vcx_scatter_add(const int32_t* idx, const void* val, int val_is_bf16, int64_t m, float scale, float* dense,
                     hipStream_t s) {
  const int grid = stream_grid(m, 256, 1024);
  if (val_is_bf16)
    hipLaunchKernelGGL(scatter_add_kernel<bf16>, dim3(grid), dim3(256), 0, s, idx, (const bf16*)val, m, scale, dense);
  else
    hipLaunchKernelGGL(scatter_add_kernel<float>, dim3(grid), dim3(256), 0, s, idx, (const float*)val, m, scale,
                       dense);
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

void vcx_psgd_orth(const void* desc, int nmat, float* P, int rank, hipStream_t s) {
  PSGD_R_DISPATCH(rank, hipLaunchKernelGGL(psgd_orth_kernel<R>, dim3(nmat), dim3(256), 0, s, (const MatDesc*)desc, P));
}

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
