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
// k_stem_fwd: block = kSGroups groups of 4 output rows (one row per wave), packed weights staged
// once, each group's 13 input rows prefetched into registers while the previous group computes;
// each wave walks its row in 32-pixel quarters with a 32 x 64 accumulator pair; epilogue rounds to
// bf16, emits per-channel (sum, sum of squares) partials of the rounded output in the [block][2][64]
// format of the BatchNorm finalize (no BN statistics pass), and stores 16-byte rows via LDS.
#include <type_traits>

#include "pde_act.h"
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
                                                  int OH, int OW, int ngroups, int total_groups) {
  __shared__ __attribute__((aligned(16))) char smem[kSInRows * kSInCols * 8 + kSC * kSWStride * 2 +
                                                   4 * 32 * 128 + 4 * 2 * kSC * 4];
  char* xin = smem;                                          // [13][230][4] bf16
  char* wp = xin + kSInRows * kSInCols * 8;                  // [64][232] bf16
  char* stage = wp + kSC * kSWStride * 2;                    // [4 waves][32 px][64 ch] bf16
  float* wstats = reinterpret_cast<float*>(stage + 4 * 32 * 128);   // [4 waves][2][64]
  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), g = l >> 5, i32 = l & 31;
  const int rgroups = (OH + kSRows - 1) / kSRows;           // 4-row groups per image
  // packed weights once per block (28 KB), reused by all of its row groups
  for (int e = t; e < kSC * kSK / 8; e += 256) {
    const int n = e / (kSK / 8), ch = e - n * (kSK / 8);
    *reinterpret_cast<uint4*>(wp + n * kSWStride * 2 + ch * 16) = reinterpret_cast<const uint4*>(Wp)[e];
  }
  // software pipeline over this block's row groups: the next group's 13 input rows are loaded into
  // registers while the current group computes from LDS.  A thread's staged pixels e = t + 256 j sit at
  // the same (row r_j, column) of every group, so their row / column split (a division), the column
  // bounds and the in-row element offset are fixed once per block; a group adds one row base
  const int ncols = 2 * OW + 6;
  constexpr int kPF = (kSInRows * kSInCols + 255) / 256;    // staged pixels per thread (<= 12)
  uint2 pf[kPF];
  int pr[kPF], poff[kPF];
  uint32_t pcol = 0;                                          // bit j: column of pixel j inside the image
#pragma unroll
  for (int j = 0; j < kPF; ++j) {
    const int e = t + 256 * j, r = e / ncols, col = e - r * ncols, iw = col - 3;
    pr[j] = r < kSInRows ? r : (1 << 20);                     // past the staged rows: never loaded
    poff[j] = r * Wd * 3 + iw * 3;
    pcol |= (iw >= 0 && iw < Wd) ? (1u << j) : 0u;
  }
  const int gbeg = blockIdx.x * ngroups, gend = min(gbeg + ngroups, total_groups);
  auto prefetch = [&](int grp) {
    const int b = grp / rgroups, ih0 = 2 * (grp - b * rgroups) * kSRows - 3;
    const bf16_t* base = X + ((ptrdiff_t)b * H + ih0) * Wd * 3;   // (row ih0, column 0) of image b
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
      const int ih = ih0 + pr[j];
      pf[j] = make_uint2(0u, 0u);
      if (((pcol >> j) & 1u) && (unsigned)ih < (unsigned)H) {
        const bf16_t* src = base + poff[j];
        pf[j].x = (uint32_t)src[0] | ((uint32_t)src[1] << 16);
        pf[j].y = (uint32_t)src[2];
      }
    }
  };
  float s_lo = 0.f, q_lo = 0.f, s_hi = 0.f, q_hi = 0.f;     // channel i32 / i32 + 32 partials
  char* st = stage + w * 32 * 128;
  if (gbeg < gend) prefetch(gbeg);
  for (int grp = gbeg; grp < gend; ++grp) {
    const int b = grp / rgroups, oh0 = (grp - b * rgroups) * kSRows;
    __syncthreads();                                         // previous group's LDS reads are done
#pragma unroll
    for (int j = 0; j < kPF; ++j) {
      const int e = t + 256 * j, r = e / ncols, col = e - r * ncols;
      if (r < kSInRows) *reinterpret_cast<uint2*>(xin + (r * kSInCols + col) * 8) = pf[j];
    }
    __syncthreads();
    if (grp + 1 < gend) prefetch(grp + 1);
    // ---- each wave: one output row, 32-pixel quarters ----
    const int oh = oh0 + w;
    if (oh < OH) {
      for (int q0 = 0; q0 < OW; q0 += 32) {
        const int ow = min(q0 + i32, OW - 1);
        f32x16 acc0 = {0.f}, acc1 = {0.f};
        // a kernel row's 6 fragments (2 image, 4 weight) are read before its 4 MFMAs (counted waits)
#pragma unroll
        for (int kh = 0; kh < 7; ++kh) {
          bf16x8 a[2], b0[2], b1[2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            a[h] = *reinterpret_cast<const bf16x8*>(xin + ((2 * w + kh) * kSInCols + 2 * ow + 4 * h + 2 * g) * 8);
            const int koff = (kh * 32 + 16 * h + 8 * g) * 2;
            b0[h] = *reinterpret_cast<const bf16x8*>(wp + i32 * kSWStride * 2 + koff);
            b1[h] = *reinterpret_cast<const bf16x8*>(wp + (i32 + 32) * kSWStride * 2 + koff);
          }
          __builtin_amdgcn_sched_barrier(0);
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            acc0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[h], b0[h], acc0, 0, 0, 0);
            acc1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[h], b1[h], acc1, 0, 0, 0);
          }
        }
        // epilogue: D reg r -> pixel row (r&3) + 8*(r>>2) + 4*g, channel i32 (+32).  The two channels
        // of a register pair are rounded by one packed convert and stored as the low / high halves
        // of that word; the statistics of the rounded values use packed adds / FMAs; only the last,
        // partial quarter of a row masks pixels
        auto epi = [&](auto FULL_) {
          constexpr bool FULL = decltype(FULL_)::value;
          pde_f2 sacc = {s_lo, s_hi}, qacc = {q_lo, q_hi};
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int px = (r & 3) + 8 * (r >> 2) + 4 * g;
            const uint32_t pk = pack_bf2(acc0[r], acc1[r]);
            pde_f2 f = {__uint_as_float(pk << 16), __uint_as_float(pk & 0xffff0000u)};
            if constexpr (!FULL) {
              const float m = q0 + px < OW ? 1.f : 0.f;
              f = f * m;
            }
            sacc += f;
            qacc = f * f + qacc;
            *reinterpret_cast<uint16_t*>(st + px * 128 + i32 * 2) = (uint16_t)pk;
            *reinterpret_cast<uint16_t*>(st + px * 128 + (i32 + 32) * 2) = (uint16_t)(pk >> 16);
          }
          s_lo = sacc.x; s_hi = sacc.y; q_lo = qacc.x; q_hi = qacc.y;
        };
        if (q0 + 32 <= OW) epi(std::true_type{});
        else epi(std::false_type{});
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
  }
  // ---- BN statistics of the block: lanes l and l^32 hold the same channels (other pixel rows) ----
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

// =================================================================================================
// k_stem_wgrad: dW[n][kh][kw][c] = sum over (b, oh, ow) of dY[b,oh,ow][n] * X[b, 2oh-3+kh, 2ow-3+kw][c].
// GEMM view M = n (64), N = packed k (224: tile t = kernel row kh), K = output pixels.  A block owns
// kSWRows output rows of one image; per row it stages dY transposed ([n][pixel], so an A fragment
// -- 8 consecutive pixels of one channel -- is one 16-byte LDS read) and the 7 input rows as
// [col][4 ch]; B fragments (8 pixels of one (kh, kw, c)) are 8 two-byte reads at a 16-byte stride.
// Wave w accumulates kernel rows kh = w and w + 4 for both 32-channel halves.  fp32 partials
// [block][64][147] are summed by k_stem_wgrad_reduce into the bf16 gradient.
// =================================================================================================
constexpr int kSWRows = 28;              // output rows per wgrad block
constexpr int kSPixStride = 160;         // bf16 per dY^T row (128 swizzled pixels + pad; 320 B)

// dY^T byte offset of (channel, pixel): the 8-pixel group index is XORed with (ch >> 3) & 7.  With the
// 320-B row stride both the transposed 2-byte stores (lanes = 8 pixels x 8 channel octets) and the
// 16-byte A-fragment reads (lanes = 32 channels at one pixel octet) hit distinct banks; the plain
// 240-B layout put every channel octet of a store on one bank (16-way, 45 M conflict cycles per
// dispatch in the round-2 counters).
__device__ __forceinline__ int dyt_off(int ch, int px) {
  return (ch * kSPixStride + ((((px >> 3) ^ ((ch >> 3) & 7)) << 3) | (px & 7))) * 2;
}

__global__ __launch_bounds__(256) void k_stem_wgrad(const bf16_t* __restrict__ X, const bf16_t* __restrict__ dY,
                                                    float* __restrict__ part, int H, int Wd, int OH, int OW) {
  __shared__ __attribute__((aligned(16))) char smem[kSC * kSPixStride * 2 + 7 * kSInCols * 8];
  char* dyt = smem;                                          // [64][160] bf16 (swizzled)
  char* xin = smem + kSC * kSPixStride * 2;                  // [7][230][4] bf16
  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6), g = l >> 5, i32 = l & 31;
  const int rblocks = (OH + kSWRows - 1) / kSWRows;
  const int b = blockIdx.x / rblocks, oh_lo = (blockIdx.x - b * rblocks) * kSWRows;
  const int oh_hi = min(oh_lo + kSWRows, OH);
  const int ntl = w < 3 ? 2 : 1;                             // kernel rows of this wave: w, w + 4
  f32x16 acc[2][2];
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int m = 0; m < 2; ++m) acc[a][m] = f32x16{0.f};
  const int npix16 = (OW + 15) / 16;
  const int ncols = 2 * (16 * npix16) + 6;                   // every column a padded pixel reads (zeros
                                                              // beyond the image: 0 * NaN must not occur)
  // software pipeline: row oh+1's global loads are in flight while row oh computes from LDS
  constexpr int kPY = (kSMaxOW * 8 + 255) / 256;             // 16-B dY pieces per thread (<= 4)
  constexpr int kPX = (7 * kSInCols + 255) / 256;            // staged input pixels per thread (<= 7)
  uint4 pf_dy[kPY];
  uint2 pf_x[kPX];
  auto prefetch = [&](int oh) {
#pragma unroll
    for (int j = 0; j < kPY; ++j) {
      const int e = t + 256 * j, px = e >> 3, c8 = e & 7;
      pf_dy[j] = make_uint4(0u, 0u, 0u, 0u);
      if (px < OW) pf_dy[j] = reinterpret_cast<const uint4*>(dY + (((size_t)b * OH + oh) * OW + px) * kSC)[c8];
    }
    const int ih0 = 2 * oh - 3;
#pragma unroll
    for (int j = 0; j < kPX; ++j) {
      const int e = t + 256 * j, r = e / ncols, col = e - r * ncols, ih = ih0 + r, iw = col - 3;
      pf_x[j] = make_uint2(0u, 0u);
      if (r < 7 && ih >= 0 && ih < H && iw >= 0 && iw < Wd) {
        const bf16_t* src = X + (((size_t)b * H + ih) * Wd + iw) * 3;
        pf_x[j].x = (uint32_t)src[0] | ((uint32_t)src[1] << 16);
        pf_x[j].y = (uint32_t)src[2];
      }
    }
  };
  if (oh_lo < oh_hi) prefetch(oh_lo);
  for (int oh = oh_lo; oh < oh_hi; ++oh) {
    __syncthreads();                                         // previous row's LDS reads are done
    // dY row -> dY^T ([n][pixel]: 8 two-byte LDS stores per 16-B piece); input rows -> [col][4 ch]
#pragma unroll
    for (int j = 0; j < kPY; ++j) {
      const int e = t + 256 * j, px = e >> 3, c8 = e & 7;
      if (px < 16 * npix16) {
        const uint32_t wv[4] = {pf_dy[j].x, pf_dy[j].y, pf_dy[j].z, pf_dy[j].w};
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          *reinterpret_cast<bf16_t*>(dyt + dyt_off(c8 * 8 + 2 * k, px)) = (bf16_t)(wv[k] & 0xffffu);
          *reinterpret_cast<bf16_t*>(dyt + dyt_off(c8 * 8 + 2 * k + 1, px)) = (bf16_t)(wv[k] >> 16);
        }
      }
    }
#pragma unroll
    for (int j = 0; j < kPX; ++j) {
      const int e = t + 256 * j, r = e / ncols, col = e - r * ncols;
      if (r < 7) *reinterpret_cast<uint2*>(xin + (r * kSInCols + col) * 8) = pf_x[j];
    }
    __syncthreads();
    if (oh + 1 < oh_hi) prefetch(oh + 1);
    for (int s16 = 0; s16 < npix16; ++s16) {
      const int p0 = 16 * s16 + 8 * g;                       // this lane group's 8 pixels
      const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(dyt + dyt_off(i32, p0));
      const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(dyt + dyt_off(i32 + 32, p0));
#pragma unroll
      for (int a = 0; a < 2; ++a) {
        if (a < ntl) {
          const int kh = w + 4 * a, kk = i32, kw = kk >> 2, c = kk & 3;
          const bf16_t* src = reinterpret_cast<const bf16_t*>(xin) + ((kh * kSInCols + 2 * p0 + kw) * 4 + c);
          bf16x8 bv;
#pragma unroll
          for (int e = 0; e < 8; ++e) bv[e] = (short)src[e * 8];   // pixels p0 + e: 2 columns = 8 bf16 apart
          acc[a][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bv, acc[a][0], 0, 0, 0);
          acc[a][1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bv, acc[a][1], 0, 0, 0);
        }
      }
    }
  }
  // partials: D reg r -> row n = (r&3) + 8*(r>>2) + 4*g (+32 m), col kk = i32 of kernel row kh
  float* out = part + (size_t)blockIdx.x * kSC * 147;
#pragma unroll
  for (int a = 0; a < 2; ++a) {
    if (a < ntl) {
      const int kh = w + 4 * a, kw = i32 >> 2, c = i32 & 3;
      if (kw < 7 && c < 3) {
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int n = (r & 3) + 8 * (r >> 2) + 4 * g + 32 * m;
            out[n * 147 + kh * 21 + kw * 3 + c] = acc[a][m][r];
          }
      }
    }
  }
}

// dW[e] = sum over blocks of part[blk][e]: block = 64 consecutive elements x 4 block slices, 16 loads
// in flight per thread (a thread per element with a serial loop over ~1000 partials was latency
// bound: 100 us for 38 MB)
__global__ __launch_bounds__(256) void k_stem_wgrad_reduce(const float* __restrict__ part, int nblk,
                                                           bf16_t* __restrict__ dW) {
  __shared__ float red[4][64];
  const int el = threadIdx.x & 63, sl = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el;
  const int ec = min(e, kSC * 147 - 1);
  float acc[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) acc[u] = 0.f;
  for (int k0 = sl; k0 < nblk; k0 += 4 * 16) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int k = k0 + 4 * u;
      acc[u] += k < nblk ? part[(size_t)k * kSC * 147 + ec] : 0.f;
    }
  }
  float s = 0.f;
#pragma unroll
  for (int u = 0; u < 16; ++u) s += acc[u];
  red[sl][el] = s;
  __syncthreads();
  if (sl == 0 && e < kSC * 147) dW[e] = f2bf((red[0][el] + red[1][el]) + (red[2][el] + red[3][el]));
}

}  // namespace

extern "C" {

int pde_stem_wgrad_blocks(int Bn, int OH) { return Bn * ((OH + kSWRows - 1) / kSWRows); }

hipError_t pde_stem_wgrad(const void* X, const void* dY, float* part, void* dW, int Bn, int H, int Wd,
                          hipStream_t st) {
  const int OH = (H - 1) / 2 + 1, OW = (Wd - 1) / 2 + 1;
  if (OW > kSMaxOW || OW < 1 || OH < 1) return hipErrorInvalidValue;
  const int nblk = pde_stem_wgrad_blocks(Bn, OH);
  hipLaunchKernelGGL(k_stem_wgrad, dim3(nblk), dim3(256), 0, st, (const bf16_t*)X, (const bf16_t*)dY, part, H, Wd,
                     OH, OW);
  hipLaunchKernelGGL(k_stem_wgrad_reduce, dim3((kSC * 147 + 63) / 64), dim3(256), 0, st, part, nblk, (bf16_t*)dW);
  return hipGetLastError();
}


constexpr int kSGroups = 7;              // 4-row groups per fwd block (weights staged once per block)

int pde_stem_stats_blocks(int Bn, int OH) { return (Bn * ((OH + kSRows - 1) / kSRows) + kSGroups - 1) / kSGroups; }

hipError_t pde_stem_fwd(const void* X, const void* W, void* Wp, void* Y, float* stats, int Bn, int H, int Wd,
                        hipStream_t st) {
  const int OH = (H - 1) / 2 + 1, OW = (Wd - 1) / 2 + 1;
  if (OW > kSMaxOW || OW < 1 || OH < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_stem_wpack, dim3((kSC * kSK + 255) / 256), dim3(256), 0, st, (const bf16_t*)W, (bf16_t*)Wp);
  hipLaunchKernelGGL(k_stem_fwd, dim3(pde_stem_stats_blocks(Bn, OH)), dim3(256), 0, st, (const bf16_t*)X,
                     (const bf16_t*)Wp, (bf16_t*)Y, stats, H, Wd, OH, OW, kSGroups, Bn * ((OH + kSRows - 1) / kSRows));
  return hipGetLastError();
}

}  // extern "C"
