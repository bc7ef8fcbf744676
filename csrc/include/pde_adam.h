// Element-wise torch.optim.Adam / AdamW update (torch/optim/adam.py:347-460 single-tensor math),
// used by the fused flat optimizers (optim.hip).
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
