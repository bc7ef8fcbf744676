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
