// Activation functions shared by the elementwise kernels and the GEMM epilogues.
#pragma once
#include <hip/hip_runtime.h>

// tanh-approximate GELU (GPT-2's gelu_new); *dgelu (optional) receives d gelu / dx
__device__ __forceinline__ float gelu_t(float x, float* dgelu) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float u = k0 * (x + k1 * x * x * x);
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * u) + 1.f);   // tanh(u), v_rcp_f32
  if (dgelu) *dgelu = 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  return 0.5f * x * (1.f + t);
}

// The same function for two values at once in the sigmoid form the GEMM epilogues use:
//   gelu(x) = 0.5 x (1 + tanh u) = x s,  s = sigmoid(2u) = 1 / (1 + 2^(-2u log2 e)),  u = k0 (x + k1 x^3)
//   gelu'(x) = s + x s (1 - s) 2u'(x),   2u'(x) = 2 k0 (1 + 3 k1 x^2)
// The polynomial / product parts are float2 arithmetic (v_pk_mul_f32 / v_pk_fma_f32 / v_pk_add_f32 on
// gfx950: two lanes' worth per VALU issue); exp2 and rcp stay one value per instruction.
typedef float pde_f2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ pde_f2 gelu2_sig(pde_f2 x, pde_f2& x2) {
  constexpr float L2E = 1.4426950408889634f, K0 = 0.7978845608028654f, K1 = 0.044715f;
  constexpr float A = -2.f * K0 * K1 * L2E, B = -2.f * K0 * L2E;      // -2u log2e = x (B + A x^2)
  x2 = x * x;
  const pde_f2 z = x * (x2 * A + B);
  pde_f2 s;
  s.x = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z.x));
  s.y = __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(z.y));
  return s;
}

// gelu of two values
__device__ __forceinline__ pde_f2 gelu2(pde_f2 x) {
  pde_f2 x2;
  return x * gelu2_sig(x, x2);
}

// gelu and gelu' of two values
__device__ __forceinline__ pde_f2 gelu2_d(pde_f2 x, pde_f2& d) {
  constexpr float K0 = 0.7978845608028654f, K1 = 0.044715f;
  pde_f2 x2;
  const pde_f2 s = gelu2_sig(x, x2);
  const pde_f2 y = x * s;
  const pde_f2 du = x2 * (6.f * K0 * K1) + 2.f * K0;                 // 2u'(x)
  d = (y - y * s) * du + s;                                          // s + x s (1 - s) 2u'
  return y;
}
