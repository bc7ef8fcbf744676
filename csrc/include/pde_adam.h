// Element-wise torch.optim.Adam / AdamW update (torch/optim/adam.py:347-460 single-tensor math),
// shared by the fused optimizer (optim.hip) and the in-kernel optimizer epilogues of the LeNet step
// (lenet_v2.hip).
#pragma once
#include <hip/hip_runtime.h>

__device__ __forceinline__ void adam_elem(float& p, float& m, float& v, float gr, float lr, float wd, int decoupled,
                                          float omb1, float omb2, float b2, float step_size, float bc2s, float eps) {
  if (wd != 0.f) {
    if (decoupled) p = p * (1.f - lr * wd);
    else gr = gr + wd * p;
  }
  m = m + omb1 * (gr - m);
  v = v * b2 + omb2 * gr * gr;
  const float denom = sqrtf(v) / bc2s + eps;
  p = p - step_size * (m / denom);
}

// Per-step constants of the update at optimizer step t (1-based).
struct AdamStep {
  float omb1, omb2, step_size, bc2s;
};
__device__ __forceinline__ AdamStep adam_step_consts(float lr, float b1, float b2, long long t) {
  AdamStep s;
  const float bc1 = 1.f - powf(b1, (float)t);
  const float bc2 = 1.f - powf(b2, (float)t);
  s.step_size = lr / bc1;
  s.bc2s = sqrtf(bc2);
  s.omb1 = 1.f - b1;
  s.omb2 = 1.f - b2;
  return s;
}
