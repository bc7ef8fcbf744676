// ResNet stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels) on bf16 MFMA, NHWC.
//
// The library path (MIOpen igemm_fwd_gtcx35 / igemm_wrw_gtcx35) took 382 + 359 us per step at
// B=256 (profiles/resnet18_w1_kernel_stats.md), 8% of the ResNet-18 step, plus a separate BN
// statistics pass.  C = 3 fits no 64-channel implicit-GEMM tile, so the stem gets its own layout:
//
//   K ordered (kh, kw, c) with c padded 3 -> 4 and kw padded 7 -> 8: one kernel row kh is a
//   32-wide K slice = two v_mfma_f32_32x32x16_bf16 steps, and the 8 K values a lane holds
//   (kw pair 2g, 2g+1 x 4 channels) are 16 CONTIGUOUS bytes of the input row staged in LDS as
//   [row][col][4 ch] -- one ds_read_b128 per A fragment, no im2col.
//   Padded K entries meet zero weights (Wp, packed once per step by k_stem_wpack).
//
// k_stem_fwd: block = 4 output rows of one image (one per wave), 13 input rows staged once;
// each wave walks its row in 32-pixel quarters with a 32 x 64 accumulator pair; epilogue rounds to
// bf16, emits per-channel (sum, sum of squares) partials of the rounded output in the [block][2][64]
// format of the BatchNorm finalize (no BN statistics pass), and stores 16-byte rows via LDS.
#include "pde_bf16.h"
#include "pde_hip.h"
#include "pde_kernels.h"

namespace {

constexpr int kSC = 64;                  // output channels
constexpr int kSK = 224;                 // packed K: 7 kh x 8 kw x 4 c
constexpr int kSWStride = 232;           // bf16 per packed weight row in LDS (464 B: conflict-free b128)
constexpr int kSRows = 4;                // output rows per block
constexpr int kSInRows = 2 * kSRows + 5; // input rows staged per block
constexpr int kSMaxOW = 112;             // widest output row supported (input width <= 224)
constexpr int kSInCols = 2 * kSMaxOW + 6;   // staged columns: iw = col - 3

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

// Wp[n][kh*32 + kw*4 + c] = W[n][kh][kw][c] (channels-last [64][7][7][3]), zero padding
__global__ void k_stem_wpack(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wp) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= kSC * kSK) return;
  const int n = e / kSK, r = e - n * kSK, kh = r >> 5, kk = r & 31, kw = kk >> 2, c = kk & 3;
  Wp[e] = (kw < 7 && c < 3) ? W[n * 147 + kh * 21 + kw * 3 + c] : (bf16_t)0;
}

__global__ __launch_bounds__(256) void k_stem_fwd(const bf16_t* __restrict__ X, const bf16_t* __restrict__ Wp,
                                                  bf16_t* __restrict__ Y, float* __restrict__ stats, int H, int Wd,
                                                  int OH, int OW) {
  __shared__ __attribute__((aligned(16))) char smem[kSInRows * kSInCols * 8 + kSC * kSWStride * 2 +
                                                   4 * 32 * 128 + 4 * 2 * kSC * 4];
  char* xin = smem;                                          // [13][230][4] bf16
  char* wp = xin + kSInRows * kSInCols * 8;                  // [64][232] bf16
  char* stage = wp + kSC * kSWStride * 2;                    // [4 waves][32 px][64 ch] bf16
  float* wstats = reinterpret_cast<float*>(stage + 4 * 32 * 128);   // [4 waves][2][64]
  const int t = threadIdx.x, l = t & 63, w = t >> 6, g = l >> 5, i32 = l & 31;
  const int rgroups = (OH + kSRows - 1) / kSRows;
  const int b = blockIdx.x / rgroups, oh0 = (blockIdx.x - b * rgroups) * kSRows;
  // ---- stage packed weights (28 KB, 16-byte loads) and the 13 input rows (zero padded) ----
  for (int e = t; e < kSC * kSK / 8; e += 256) {
    const int n = e / (kSK / 8), ch = e - n * (kSK / 8);
    *reinterpret_cast<uint4*>(wp + n * kSWStride * 2 + ch * 16) = reinterpret_cast<const uint4*>(Wp)[e];
  }
  // input rows, zero padded, [iw][3] -> [col][4] (measured: 2-byte global loads here beat 4-byte
  // pair loads + scattered 2-byte LDS writes + a zeroing pass, 228 vs ~270 us per step at B=256)
  const int ih0 = 2 * oh0 - 3, ncols = 2 * OW + 6;
  for (int e = t; e < kSInRows * ncols; e += 256) {
    const int r = e / ncols, col = e - r * ncols, ih = ih0 + r, iw = col - 3;
    uint2 v = make_uint2(0u, 0u);
    if (ih >= 0 && ih < H && iw >= 0 && iw < Wd) {
      const bf16_t* src = X + (((size_t)b * H + ih) * Wd + iw) * 3;
      v.x = (uint32_t)src[0] | ((uint32_t)src[1] << 16);
      v.y = (uint32_t)src[2];
    }
    *reinterpret_cast<uint2*>(xin + (r * kSInCols + col) * 8) = v;
  }
  __syncthreads();
  // ---- each wave: one output row, 32-pixel quarters ----
  const int oh = oh0 + w;
  float s_lo = 0.f, q_lo = 0.f, s_hi = 0.f, q_hi = 0.f;     // channel i32 / i32 + 32 partials
  char* st = stage + w * 32 * 128;
  if (oh < OH) {
    for (int q0 = 0; q0 < OW; q0 += 32) {
      const int ow = min(q0 + i32, OW - 1);
      f32x16 acc0 = {0.f}, acc1 = {0.f};
#pragma unroll
      for (int kh = 0; kh < 7; ++kh) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x8 a = *reinterpret_cast<const bf16x8*>(xin + ((2 * w + kh) * kSInCols + 2 * ow + 4 * h + 2 * g) * 8);
          const int koff = (kh * 32 + 16 * h + 8 * g) * 2;
          const bf16x8 b0 = *reinterpret_cast<const bf16x8*>(wp + i32 * kSWStride * 2 + koff);
          const bf16x8 b1 = *reinterpret_cast<const bf16x8*>(wp + (i32 + 32) * kSWStride * 2 + koff);
          acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b0, acc0, 0, 0, 0);
          acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b1, acc1, 0, 0, 0);
        }
      }
      // epilogue: D reg r -> pixel row (r&3) + 8*(r>>2) + 4*g, channel i32 (+32)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int px = (r & 3) + 8 * (r >> 2) + 4 * g;
        const bool valid = q0 + px < OW;
        const bf16_t v0 = f2bf(acc0[r]), v1 = f2bf(acc1[r]);
        const float f0 = bf2f(v0), f1 = bf2f(v1);
        if (valid) {
          s_lo += f0; q_lo += f0 * f0;
          s_hi += f1; q_hi += f1 * f1;
        }
        *reinterpret_cast<bf16_t*>(st + px * 128 + i32 * 2) = v0;
        *reinterpret_cast<bf16_t*>(st + px * 128 + (i32 + 32) * 2) = v1;
      }
      // the stage is private to this wave: wave-level LDS ordering is enough
      __builtin_amdgcn_s_waitcnt(0xC07F);            // lgkmcnt(0)
      __builtin_amdgcn_wave_barrier();
      const size_t rowbase = (((size_t)b * OH + oh) * OW + q0) * kSC;
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = l + 64 * u, px = c >> 3, part = c & 7;
        if (q0 + px < OW)
          reinterpret_cast<uint4*>(Y + rowbase + (size_t)px * kSC)[part] =
              *reinterpret_cast<const uint4*>(st + px * 128 + part * 16);
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_wave_barrier();
    }
  }
  // ---- BN statistics: lanes l and l^32 hold the same channels (other pixel rows) ----
  s_lo += __shfl_xor(s_lo, 32, 64);
  q_lo += __shfl_xor(q_lo, 32, 64);
  s_hi += __shfl_xor(s_hi, 32, 64);
  q_hi += __shfl_xor(q_hi, 32, 64);
  if (stats) {
    if (g == 0) {
      wstats[(w * 2 + 0) * kSC + i32] = s_lo;
      wstats[(w * 2 + 0) * kSC + i32 + 32] = s_hi;
      wstats[(w * 2 + 1) * kSC + i32] = q_lo;
      wstats[(w * 2 + 1) * kSC + i32 + 32] = q_hi;
    }
    __syncthreads();
    if (t < 2 * kSC) {
      const int row = t >> 6, ch = t & 63;
      float acc = 0.f;
#pragma unroll
      for (int ww = 0; ww < 4; ++ww) acc += wstats[(ww * 2 + row) * kSC + ch];
      stats[(size_t)blockIdx.x * 2 * kSC + row * kSC + ch] = acc;
    }
  }
}

}  // namespace

extern "C" {

int pde_stem_stats_blocks(int Bn, int OH) { return Bn * ((OH + kSRows - 1) / kSRows); }

hipError_t pde_stem_fwd(const void* X, const void* W, void* Wp, void* Y, float* stats, int Bn, int H, int Wd,
                        hipStream_t st) {
  const int OH = (H - 1) / 2 + 1, OW = (Wd - 1) / 2 + 1;
  if (OW > kSMaxOW || OW < 1 || OH < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stem_wpack, dim3((kSC * kSK + 255) / 256), dim3(256), 0, st, (const bf16_t*)W, (bf16_t*)Wp);
  hipLaunchKernelGGL(k_stem_fwd, dim3(pde_stem_stats_blocks(Bn, OH)), dim3(256), 0, st, (const bf16_t*)X,
                     (const bf16_t*)Wp, (bf16_t*)Y, stats, H, Wd, OH, OW);
  return hipGetLastError();
}

}  // extern "C"
