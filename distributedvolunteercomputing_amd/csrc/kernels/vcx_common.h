// Shared device helpers for the gfx950 (CDNA4, MI355X) kernels of this package.
//
// Conventions used by every kernel file:
//   * wave64: all cross-lane reductions are over 64 lanes (never 32).
//   * bf16 is clang's native __bf16; f32->bf16 lowers to v_cvt_pk_bf16_f32 (RNE) on gfx950.
//   * memory-bound kernels move 16 B per lane per access (bf16x8 / f32x4).
//   * launchers are plain C++ functions taking raw device pointers + hipStream_t, so the
//     same entry points serve the torch binding, graph capture and the C++ tests.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace vcx {

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef short s16x8 __attribute__((ext_vector_type(8)));

constexpr int kWave = 64;
constexpr int kNumCU = 256;

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `scratch` needs NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* scratch) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += scratch[i];
  return r;
}

template <int NT>
__device__ __forceinline__ float block_max(float v, float* scratch) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  __syncthreads();
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, scratch[i]);
  return r;
}

// Grid size for a grid-stride memory-bound kernel: enough blocks to fill 256 CUs several
// times over without launching millions of tiny blocks.
inline int stream_grid(int64_t work_items, int per_block, int max_blocks = 256 * 8) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

}  // namespace vcx

#define VCX_LAUNCH_CHECK() (void)hipGetLastError()
