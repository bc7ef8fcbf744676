// Shared layout helpers of the LeNet (toy CNN) kernels (device + host).
#pragma once
#include <hip/hip_runtime.h>

constexpr int kPdeWpFloats = 2 * 72 * 256;   // packed conv2 weight of k_conv_fwd2 (two 72 KB co-halves)

// conv2.weight [50][20][5][5] element e -> index in the packed layout read by k_conv_fwd2
// (lenet_v2.hip): Wp[ct][cotile][kq][co16][132], k' = (kh*5+kw)*20 + ci at k-step k'>>2, lane group k'&3.
__host__ __device__ __forceinline__ int pde_lenet_wp_index(int e) {
  const int co = e / 500, k = e - co * 500, ci = k / 25, tap = k - ci * 25;
  const int kp = tap * 20 + ci, s = kp >> 2, kq = kp & 3;
  return (co >> 5) * (72 * 256) + ((((co >> 4) & 1) * 4 + kq) * 16 + (co & 15)) * 132 + s;
}
