// Common CDNA4 (gfx950) helpers for the framework's HIP kernels.
//
// Wave64 everywhere; MFMA fragment conventions (cdna_hip_programming.md §3):
//   v_mfma_f32_16x16x4_f32 : lane l holds A[i=l&15][k=l>>4], B[k=l>>4][j=l&15];
//                            C/D reg r -> row (l>>4)*4+r, col l&15.
//   v_mfma_f32_32x32x2_f32 : lane l holds A[i=l&31][k=l>>5], B[k=l>>5][j=l&31];
//                            C/D reg r -> row (r&3)+8*(r>>2)+4*(l>>5), col l&31.
// Because the K index of a fragment is private to the lane group, any per-group permutation of
// K that is applied identically to A and B gives the same product.  The kernels use that to load
// 4 consecutive K values per lane with one 16-byte load ("lane-contiguous K").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PDE_WAVE 64

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

__device__ __forceinline__ f32x4 mfma16x16x4(float a, float b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x16 mfma32x32x2(float a, float b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, c, 0, 0, 0);
}

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

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }

// Bijective XCD-aware remap of a linear block id (cdna_hip_programming.md §5 "XCD swizzle must be
// bijective"): blocks that the dispatcher deals round-robin to the same XCD get contiguous ids.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

#define PDE_HIP_CHECK(expr)                                                              \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) return _e;                                                     \
  } while (0)
