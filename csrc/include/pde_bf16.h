// bf16 helpers for the transformer / ResNet kernels (gfx950).
//
// bf16 is carried as raw uint16 in memory.  f32 -> bf16 uses the compiler's __bf16 conversion, which
// lowers to v_cvt_pk_bf16_f32 (round-to-nearest-even, two values per instruction) on gfx950.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

typedef uint16_t bf16_t;
typedef short bf16x8 __attribute__((ext_vector_type(8)));     // MFMA A/B fragment (4 VGPRs)
typedef short bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2v __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float bf2f(uint32_t h) { return __uint_as_float(h << 16); }
__device__ __forceinline__ float bf_lo(uint32_t w) { return __uint_as_float(w << 16); }
__device__ __forceinline__ float bf_hi(uint32_t w) { return __uint_as_float(w & 0xffff0000u); }

__device__ __forceinline__ uint32_t pack_bf2(float a, float b) {
  bf16x2v v;
  v[0] = (__bf16)a;
  v[1] = (__bf16)b;
  return __builtin_bit_cast(uint32_t, v);
}
__device__ __forceinline__ bf16_t f2bf(float a) { return (bf16_t)(pack_bf2(a, 0.f) & 0xffffu); }

// 4 bf16 <-> 4 floats (one 8-byte access)
__device__ __forceinline__ void unpack4(uint2 w, float* f) {
  f[0] = bf_lo(w.x); f[1] = bf_hi(w.x); f[2] = bf_lo(w.y); f[3] = bf_hi(w.y);
}
__device__ __forceinline__ uint2 pack4(const float* f) { return make_uint2(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3])); }

// 8 bf16 <-> 8 floats (one 16-byte access)
__device__ __forceinline__ void unpack8(uint4 w, float* f) {
  f[0] = bf_lo(w.x); f[1] = bf_hi(w.x); f[2] = bf_lo(w.y); f[3] = bf_hi(w.y);
  f[4] = bf_lo(w.z); f[5] = bf_hi(w.z); f[6] = bf_lo(w.w); f[7] = bf_hi(w.w);
}
__device__ __forceinline__ uint4 pack8(const float* f) {
  return make_uint4(pack_bf2(f[0], f[1]), pack_bf2(f[2], f[3]), pack_bf2(f[4], f[5]), pack_bf2(f[6], f[7]));
}

