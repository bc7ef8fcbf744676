// LeNet training step, second generation (the reference "toy CNN", /root/reference/mnist/main.py:130-147).
//
// Differences from lenet.hip's F1 (measured in-step with tools/lenet_phases.py, profiles/lenet_phases_*.md):
//  * the batch is PREFETCHED: the previous step gathered its sampler rows into Xb (double-buffered by
//    step parity, chosen on the host at launch/capture time), so the kernel starts with ONE dependent
//    global load instead of counter -> index -> image (0.9 us of chain + 3.4 us to the first barrier);
//  * the conv2 weight slice (72 KB per co-half) is staged by LDS-DMA (global_load_lds_dwordx4, 9 per
//    wave, issued after the image loads) while conv1 computes: no 64-VGPR register staging that the
//    compiler sank past conv1 (2.5 us of exposed weight latency), and no LDS write pass;
//  * 8 waves per block: conv1 tiles (v_mfma_f32_32x32x2_f32, pooling on the accumulator rows) spread
//    over 8 waves, conv2 as one 16x16 output tile per wave on v_mfma_f32_16x16x4_f32 over the full
//    K = 500 (no K-split partial sums, no LDS reduction); the A operand comes from LDS by ds_read_b128
//    (4 k-steps per read), the B operand (conv1 output im2col) by conflict-free ds_read_b32: 4x4-pixel
//    output tiles with a channel stride of 144 floats (== 16 mod 32 banks) put the two K-lane groups
//    of each 32-lane half on disjoint bank sets;
//  * bias + ReLU + 2x2 max-pool (first maximum in scan order, as ATen) on the accumulator registers with
//    lane shuffles (pixel neighbours are lanes ^1 / ^4 / ^5 of a 4x4 tile);
//  * P1 / A1 (conv1 pooled output + argmax codes, kept for backward) are written from LDS right after
//    the conv1 -> conv2 barrier (split between the two co-half blocks): behind the LDS-DMA wait, so no
//    store delays it, and they drain under conv2 instead of at the kernel tail.
//
// Packed conv2 weight ("Wp"), written by the optimizer's repack epilogue (optim.hip, pack mode 2):
//   Wp[ct][cotile][kq][co16][132]  (ct = co >> 5, cotile = (co >> 4) & 1, co16 = co & 15)
//   holding W2[co][ci][kh][kw] at k-step s = k' >> 2, kq = k' & 3, k' = (kh*5 + kw)*20 + ci;
//   rows are 132 floats (125 k-steps + zero pad; 528 B, a multiple of 16 B: co rows 4 banks apart ->
//   the b128 A reads are conflict-free); each co-half region is padded to 72 KB = 72 LDS-DMA
//   wave-instructions (9 per wave, a compile-time count, so the compiler's vmcnt bookkeeping stays exact).
#include "pde_hip.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "pde_kernels.h"
#include "pde_lenet.h"
#include "pde_peer_dev.h"

namespace {

constexpr int kImg = 784, kP1 = 2880, kFeat = 800;
constexpr int kRowS = 132;
constexpr int kWpHalf = 72 * 256;            // floats per co-half region (72 KB)
constexpr int kL_W = 0;
constexpr int kL_XS = kWpHalf;               // [20][144] pooled conv1 output
constexpr int kL_CODE = kL_XS + kP1;         // [20][144] uint8 argmax codes (720 floats)
constexpr int kImgRow = 48;                  // padded image row (28 -> 48 floats: rows 16 banks apart)
constexpr int kL_IMG = kL_CODE + 720;        // [28][48]
constexpr int kL_W1 = kL_IMG + 28 * kImgRow; // conv1 weight [500] + bias [20] (+pad)
constexpr int kL_TOT = kL_W1 + 528;          // 23904 floats = 93 KB

#define PMARK(ph)                                                                             \
  do {                                                                                        \
    if constexpr (PROF) {                                                                     \
      if (threadIdx.x == 0)                                                                   \
        prof[((size_t)blockIdx.y * gridDim.x + blockIdx.x) * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                         \
  } while (0)

template <bool PROF, bool VALU1>
__global__ __launch_bounds__(512) void k_conv_fwd2(const float* __restrict__ Xb, const float* __restrict__ w1,
                                                   const float* __restrict__ b1, const float* __restrict__ Wp,
                                                   const float* __restrict__ b2, float* __restrict__ P1,
                                                   uint8_t* __restrict__ A1, float* __restrict__ P2,
                                                   uint8_t* __restrict__ A2, float* __restrict__ zero_ptr, int zero_n,
                                                   unsigned long long* __restrict__ prof) {
  constexpr bool conv1_valu = VALU1;
  __shared__ __attribute__((aligned(16))) float smem[kL_TOT];
  const int b = blockIdx.x, ct = blockIdx.y, t = threadIdx.x, l = t & 63, w = t >> 6;
  PMARK(0);
  // ---- phase 0: register loads first (image, conv1 weights, this wave's conv2 biases) ----
  const int cotile = w >> 2, pxt = w & 3, kq = l >> 4, j = l & 15;
  const int co_base = ct * 32 + cotile * 16 + kq * 4;          // + r: the accumulator row's channel
  float4 xv, wv;
  float bv1;
  float bias2[4];
  float4 wr[9];
  if constexpr (conv1_valu) {
    // EVERY global load before conv1 is inline asm, the conv2 weight image (9 x 16 B per lane) issued
    // right behind the image and conv1 weights, so the weights are in flight from the block start;
    // hipcc never sees these loads, so none of its vmcnt waits can drain the weights early -- the
    // first three are retired by the explicit vmcnt(9), the weights by a vmcnt(0) after conv1
    const float* xsrc = Xb + (size_t)b * kImg + 4 * min(t, kImg / 4 - 1);
    const float* w1src = w1 + 4 * min(t, 124);
    const float* b1src = b1 + min(t, 19);
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(xv) : "v"(xsrc) : "memory");
    asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(wv) : "v"(w1src) : "memory");
    asm volatile("global_load_dword %0, %1, off" : "=v"(bv1) : "v"(b1src) : "memory");
    const float* wsrc = Wp + (size_t)ct * kWpHalf + w * 256 + l * 4;
#pragma unroll
    for (int i = 0; i < 9; ++i)
      asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(wr[i]) : "v"(wsrc + i * 8 * 256) : "memory");
    asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
  } else {
    xv = reinterpret_cast<const float4*>(Xb + (size_t)b * kImg)[min(t, kImg / 4 - 1)];
    wv = reinterpret_cast<const float4*>(w1)[min(t, 124)];
    bv1 = b1[min(t, 19)];
#pragma unroll
    for (int r = 0; r < 4; ++r) bias2[r] = b2[min(co_base + r, 49)];
  }
  if (t < kImg / 4) reinterpret_cast<float4*>(smem + kL_IMG + (t / 7) * kImgRow)[t % 7] = xv;
  if (t < 125) reinterpret_cast<float4*>(smem + kL_W1)[t] = wv;
  if (t < 20) smem[kL_W1 + 500 + t] = bv1;
  // ---- then the conv2 weight image: 72 x 1 KB, exactly 9 per wave.  conv1_valu: into registers
  // (issued above), written to LDS after conv1 (the LDS-DMA fill ran ~4.6 us from the block start,
  // longer than the VALU conv1); else by LDS-DMA, which lands under the 3.7 us MFMA conv1 ----
  {
    const float* wsrc = Wp + (size_t)ct * kWpHalf;
    if constexpr (!conv1_valu) {
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        const int c = w + 8 * i;
        __builtin_amdgcn_global_load_lds(wsrc + c * 256 + l * 4, smem + kL_W + c * 256, 16, 0, 0);
      }
    }
  }
  __builtin_amdgcn_sched_barrier(0);
  // gradient-buffer zeroing (atomic targets of the backward) drains while conv1 computes
  if (zero_ptr) {
    const int nb = gridDim.x * gridDim.y, bid = ct * gridDim.x + b;
    for (int i = bid * 512 + t; i < zero_n; i += nb * 512) zero_ptr[i] = 0.f;
  }
  // barrier without draining the LDS-DMA (a __syncthreads() would wait vmcnt(0))
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  PMARK(1);
  // ---- phase 1: conv1 (1->20, 5x5) + bias + ReLU + 2x2 max-pool on the VALU ----
  // 480 threads: thread = (channel c, pooled row ph, half of the row): a 6 x 16 input window in
  // registers (24 ds_read_b128), the channel's 25 weights, then 6 pooled outputs x 4 sub-positions x
  // 25 taps = 600 FMAs from registers.  (The 32x32x2 f32 MFMA form padded 20 channels to 32 and 25
  // taps to 26 -- 1.66x the FMAs at the same per-SIMD f32 rate -- and took 3.7 us of the block.)
  if constexpr (conv1_valu) {
    const float* xin = smem + kL_IMG;
    const float* w1s = smem + kL_W1;
    float* xs = smem + kL_XS;
    uint8_t* codes = reinterpret_cast<uint8_t*>(smem + kL_CODE);
    if (t < 480) {
      const int c = t / 24, rem = t - c * 24, ph = rem >> 1, hf = rem & 1;
      // the window as column PAIRS, so the two horizontal sub-positions (dx = 0, 1) of a pooling window
      // run as one packed FMA (v_pk_fma_f32: the f32 VALU's full rate, half the issue slots of
      // scalar FMAs); odd pairs (x[2i+1], x[2i+2]) are built once per row from the even ones
      typedef float f2v __attribute__((ext_vector_type(2)));
      f2v ev[6][8];
#pragma unroll
      for (int r = 0; r < 6; ++r)
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const float4 v4 = *reinterpret_cast<const float4*>(xin + (2 * ph + r) * kImgRow + 12 * hf + 4 * k);
          ev[r][2 * k] = f2v{v4.x, v4.y};
          ev[r][2 * k + 1] = f2v{v4.z, v4.w};
        }
      auto pr = [&](int r, int i) -> f2v {       // (x[r][i], x[r][i + 1]), i compile-time
        return (i & 1) ? f2v{ev[r][i >> 1].y, ev[r][(i >> 1) + 1].x} : ev[r][i >> 1];
      };
      float wt[25];
#pragma unroll
      for (int k = 0; k < 25; ++k) wt[k] = w1s[c * 25 + k];
      const float bch = w1s[500 + c];
      // a[pw][dy] = (sub-position (dy, 0), (dy, 1)); each output's FMA chain runs kh-major, kw-minor as
      // the scalar form did (bit-identical sums)
      f2v a[6][2];
#pragma unroll
      for (int pw = 0; pw < 6; ++pw) a[pw][0] = a[pw][1] = f2v{0.f, 0.f};
#pragma unroll
      for (int kh = 0; kh < 5; ++kh)
#pragma unroll
        for (int pw = 0; pw < 6; ++pw)
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            const f2v wv2 = f2v{wt[kh * 5 + kw], wt[kh * 5 + kw]};
            a[pw][0] = __builtin_elementwise_fma(pr(kh, 2 * pw + kw), wv2, a[pw][0]);
            a[pw][1] = __builtin_elementwise_fma(pr(kh + 1, 2 * pw + kw), wv2, a[pw][1]);
          }
#pragma unroll
      for (int pw = 0; pw < 6; ++pw) {
        const float qv[4] = {a[pw][0].x, a[pw][0].y, a[pw][1].x, a[pw][1].y};
        float best = 0.f;
        int code = 0;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const float v = fmaxf(qv[q] + bch, 0.f);
          if (q == 0 || v > best) {            // first maximum in scan order (ATen)
            best = v;
            code = q;
          }
        }
        const int pq = ph * 12 + 6 * hf + pw;
        xs[c * 144 + pq] = best;
        codes[c * 144 + pq] = (uint8_t)code;
      }
    }
  } else {
  // ---- phase 1: conv1 (1->20, 5x5) + bias + ReLU + 2x2 max-pool on v_mfma_f32_32x32x2_f32 ----
  // C[m][ch] = sum_tap im2col[m][tap] * W1[ch][tap], m = 4 * pooled_pos + (dy*2+dx): accumulator rows
  // 4g..4g+3 are the 4 sub-positions of one pooled position -> pooled in registers.  (Measured and
  // rejected: the transposed C[ch][m] with the pool as a max over lanes -- its 48 lane shuffles per
  // tile lower to LDS permutes and made this phase 6.6 us instead of 3.6.)
  {
    const float* xin = smem + kL_IMG;
    const float* w1s = smem + kL_W1;
    float* xs = smem + kL_XS;
    uint8_t* codes = reinterpret_cast<uint8_t*>(smem + kL_CODE);
    const int ch = l & 31, hi = l >> 5;
    const float chm = ch < 20 ? 1.f : 0.f;
    float wb[13];
#pragma unroll
    for (int s2 = 0; s2 < 13; ++s2) {
      const int tap = 2 * s2 + hi;
      wb[s2] = (tap < 25) ? w1s[min(ch, 19) * 25 + min(tap, 24)] * chm : 0.f;
    }
    const float bch = w1s[500 + min(ch, 19)];
#pragma unroll
    for (int it = 0; it < 3; ++it) {
      const int tile = w + 8 * it;
      if (tile < 18) {
        const int m = tile * 32 + ch, pp = m >> 2, sub = m & 3;
        const float* xa = xin + (2 * (pp / 12) + (sub >> 1)) * kImgRow + 2 * (pp % 12) + (sub & 1);
        float av[13];
#pragma unroll
        for (int s2 = 0; s2 < 13; ++s2) {
          const int t0 = 2 * s2, t1 = min(2 * s2 + 1, 24);
          av[s2] = hi ? xa[(t1 / 5) * kImgRow + t1 % 5] : xa[(t0 / 5) * kImgRow + t0 % 5];
        }
        f32x16 acc = {0.f};
#pragma unroll
        for (int s2 = 0; s2 < 13; ++s2) acc = mfma32x32x2(av[s2], wb[s2], acc);
        if (ch < 20) {
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int pq = tile * 8 + 2 * g + hi;          // pooled position of registers 4g..4g+3
            float best = fmaxf(acc[4 * g] + bch, 0.f);
            int code = 0;
#pragma unroll
            for (int q = 1; q < 4; ++q) {
              const float v = fmaxf(acc[4 * g + q] + bch, 0.f);
              if (v > best) { best = v; code = q; }
            }
            xs[ch * 144 + pq] = best;
            codes[ch * 144 + pq] = (uint8_t)code;
          }
        }
      }
    }
  }
  }   // conv1_valu
  if constexpr (conv1_valu) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#pragma unroll
    for (int i = 0; i < 9; ++i) *reinterpret_cast<float4*>(smem + kL_W + (w + 8 * i) * 256 + l * 4) = wr[i];
    // the conv2 biases are needed only by the epilogue: loaded now, they land under conv2
#pragma unroll
    for (int r = 0; r < 4; ++r) bias2[r] = b2[min(co_base + r, 49)];
  }
  PMARK(2);
  // conv1 output visible + this wave's LDS-DMA landed, then every wave's (barrier)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  PMARK(3);
  // ---- P1 / A1 for backward (this block's 10 channels): issued now, they drain under conv2 ----
  if (t < 360) {
    const int c0 = ct * 10 * 144;
    // non-temporal: read again only by the conv backward three kernels later, so these 1.8 MB are
    // streamed out instead of sitting dirty in the XCD L2s for the end-of-kernel write-back
    typedef float nt_f4 __attribute__((ext_vector_type(4)));
    __builtin_nontemporal_store(reinterpret_cast<const nt_f4*>(smem + kL_XS + c0)[t],
                                reinterpret_cast<nt_f4*>(P1 + (size_t)b * kP1 + c0) + t);
    __builtin_nontemporal_store(
        reinterpret_cast<const uint32_t*>(reinterpret_cast<const uint8_t*>(smem + kL_CODE) + c0)[t],
        reinterpret_cast<uint32_t*>(A1 + (size_t)b * kP1 + c0) + t);
  }
  // ---- phase 2: conv2 (20->50, 5x5): wave = (co tile of 16, 4x4 pixel tile), K = 500 ----
  const int oh = (pxt >> 1) * 4 + (j >> 2), ow = (pxt & 1) * 4 + (j & 3);
  f32x4 acc = {0.f};
  {
    const float* wa = smem + kL_W + ((cotile * 4 + kq) * 16 + j) * kRowS;   // A: W[co = j][k-steps], b128 reads
    const float* xb = smem + kL_XS + kq * 144 + oh * 12 + ow;             // B: im2col[k][px]
#pragma unroll
    for (int u = 0; u < 32; ++u) {
      const float4 a4 = *reinterpret_cast<const float4*>(wa + 4 * u);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int s = 4 * u + e;
        if (s < 125) {
          const int tap = s / 5, kh = tap / 5, kw = tap % 5, cib = 4 * (s % 5);
          const float bv = xb[cib * 144 + kh * 12 + kw];
          acc = mfma16x16x4(e == 0 ? a4.x : e == 1 ? a4.y : e == 2 ? a4.z : a4.w, bv, acc);
        }
      }
    }
  }
  PMARK(4);
  // ---- epilogue: bias + ReLU + 2x2 max-pool across lanes (^1 = dx, ^4 = dy), P2 / A2 ----
  {
    const bool anchor = (j & 5) == 0;                  // top-left pixel of a pooling window
    const int ph = oh >> 1, pw = ow >> 1;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float v = fmaxf(acc[r] + bias2[r], 0.f);
      const float v1 = __shfl_xor(v, 1, 64), v4 = __shfl_xor(v, 4, 64), v5 = __shfl_xor(v, 5, 64);
      float best = v;
      int code = 0;
      if (v1 > best) { best = v1; code = 1; }
      if (v4 > best) { best = v4; code = 2; }
      if (v5 > best) { best = v5; code = 3; }
      const int co = co_base + r;
      if (anchor && co < 50) {
        const size_t o = (size_t)b * kFeat + co * 16 + ph * 4 + pw;
        P2[o] = best;
        A2[o] = (uint8_t)code;
      }
    }
  }
  PMARK(5);
}

// Batch prefetch: rows of sampler batch (*ctr % nbatches) (or batch 0 without a counter) gathered
// into Xdst [B][784] / Ydst [B] / rows_dst [B]; indices past the end of idx are clamped (the ragged
// tail batch).  One wave per row, 4 rows per 256-thread block.
__device__ __forceinline__ void gather_rows(const float* __restrict__ X, const long long* __restrict__ labels,
                                            const int* __restrict__ idx, int n_idx, const long long* __restrict__ ctr,
                                            int nbatches, int B, float* __restrict__ Xdst, long long* __restrict__ Ydst,
                                            int* __restrict__ rows_dst, int gblock) {
  const int l = threadIdx.x & 63, r = gblock * 4 + (threadIdx.x >> 6);
  if (r >= B) return;
  const long long batch = ctr ? (*ctr % nbatches) : 0;
  const int src = idx ? idx[min(batch * B + r, (long long)n_idx - 1)] : r;
  const float4* s4 = reinterpret_cast<const float4*>(X + (size_t)src * kImg);
  float4* d4 = reinterpret_cast<float4*>(Xdst + (size_t)r * kImg);
  float4 v[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) v[i] = s4[min(l + 64 * i, kImg / 4 - 1)];
#pragma unroll
  for (int i = 0; i < 4; ++i)
    if (l + 64 * i < kImg / 4) d4[l + 64 * i] = v[i];
  if (l == 0) {
    if (Ydst) Ydst[r] = labels[src];
    if (rows_dst) rows_dst[r] = src;
  }
}

__global__ __launch_bounds__(256) void k_gather(const float* __restrict__ X, const long long* __restrict__ labels,
                                                const int* __restrict__ idx, int n_idx,
                                                const long long* __restrict__ ctr, int nbatches, int B,
                                                float* __restrict__ Xdst, long long* __restrict__ Ydst,
                                                int* __restrict__ rows_dst) {
  gather_rows(X, labels, idx, n_idx, ctr, nbatches, B, Xdst, Ydst, rows_dst, blockIdx.x);
}

// =================================================================================================
// Conv backward v2.  Two block roles of 512 threads, INTERLEAVED in dispatch order (W, D, W, D, ...)
// and sized so that at B = 128 all 512 blocks are co-resident (< 64 KB LDS -> 2 per CU on 256 CUs):
// the first generation's D blocks (60 KB, 769 blocks) waited ~7 us for W blocks to leave.
//   role W  (ig, kp): conv2 wgrad|bgrad over an image group (G = ceil(B/16) images, 16 groups) for a
//           32-column k slice, v_mfma_f32_16x16x4_f32, A = pooled gradient scattered by the argmax
//           codes on the fly, B = im2col of P1 (ones column k = 500 -> bias gradient).  slab_stride > 0:
//           group ig writes its partial into gradient replica ig (plain stores, deterministic; the
//           optimizer folds the 16 replicas); slab_stride == 0: float atomics into the gradient.
//           Side jobs: block w prefetches half (w & 1) of row (w >> 1) of the NEXT batch into the other
//           parity's buffers (counter -> index -> image; the waits land after the MFMA loop), block 0
//           folds the head's per-row loss / hit into the device meters.
//   role D  (image b, half h of 10 input channels): conv2 dgrad in two passes of 5 channels
//           (T[125 k][64 px] on v_mfma_f32_32x32x2_f32, A = W2 from registers), col2im as an LDS
//           gather + ReLU mask of P1, conv1 wgrad|bgrad on v_mfma_f32_16x16x4_f32 with the unpooled
//           gradient produced on the fly from dP1 and the maxpool-1 codes, one atomic per output into
//           replica (b % c1_nrep).  Synchronises through LDS only (raw s_barrier + lgkmcnt(0)).
// LDS layouts are padded so every hot access is bank-conflict free (SQ_LDS_BANK_CONFLICT was 3.7 M
// cycles per step before: 16-way dY2 scatter writes, 4-way gradient / code reads in W, 8-way dP1):
//   W: pooled gradient rows of 20 floats per channel (float2 reads: lanes co*20 and co*20+2 on
//      disjoint bank pairs), argmax code rows of 20 bytes (5 dwords), P1 slice [3][144];
//   D: dY2 [50][64] written in gather order from global loads, dP1 rows of 145 floats and A1 code rows
//      of 148 bytes (co-prime-ish strides across the 16 channel lanes), conv1-wgrad partials rows of 36.
// =================================================================================================
constexpr int kWImgs = 8;
constexpr int kWG = 0, kWC = 1000, kWP = 1250;     // per image: grad [50][20] | codes [50][20 B] | P1 [3][144]
constexpr int kWImgStride = kWP + 432;             // 1682 floats
constexpr int kD_DY2 = 0;                          // [50][64] dY2 (later conv1-wgrad partials [4][16][36])
constexpr int kD_T = 3200;                         // [128][64] dgrad T of one pass
constexpr int kD_P1 = kD_T + 8192;                 // [10][144] P1 of the half
constexpr int kD_C1 = kD_P1 + 1440;                // [10][148 B] A1 codes (370 floats)
constexpr int kD_X = kD_C1 + 370;                  // [784] image
constexpr int kD_DP1 = kD_X + kImg;                // [10][145] dP1 (ReLU-masked)
constexpr int kD_TOT = kD_DP1 + 1450;              // 15436 floats
constexpr int kW_TOT = kWImgs * kWImgStride + 160; // 13616 floats
constexpr int kBwd2Lds = (kD_TOT > kW_TOT ? kD_TOT : kW_TOT) + 20;   // + meter scratch, flags, peer words
constexpr int kL_FLAG = kBwd2Lds - 20;             // block-uniform flags (last-arriver decisions)
constexpr int kL_PEER = kBwd2Lds - 18;             // two words for the peer protocol (fused all-reduce)

// Deterministic gradient reduction + in-kernel optimizer (see the role comments above k_conv_bwd2).
constexpr int kNIG = 16;                           // W image groups (= conv2 wgrad slabs)
constexpr int kSlab = 25088;                       // floats per slab: weight [50][500] | pad | bias [50] at 25024
constexpr int kSlabBias = 25024;
constexpr int kC1Rep = 576;                        // int64 per conv1 replica: weight [20][25] | bias [20] at 512
                                                   // (the layout of the conv1 slots of the flat gradient buffer)
constexpr int kC1NRep = 16;
constexpr float kC1Scale = 1099511627776.f;        // 2^40 fixed point for the order-free int64 sums
constexpr int kC1BadSlot = 511;                    // replica 0, unused weight slot: non-finite partial count
constexpr int kC1Img = 520;                        // ext mode: floats per image partial (2 halves x 10 ch x 26)
constexpr double kC1InvScale = 1.0 / 1099511627776.0;
enum { kTickD = 16, kTicks = 32 };        // [0, 16): per-k-slice W tickets, [16]: D blocks

struct Bwd2Opt {
  float* slab;                 // [16][kSlab] conv2 wgrad partials (write-through stores)
  long long* c1rep;            // [16][kC1Rep] conv1 wgrad partials, fixed point (zero at rest; fold mode)
  float* c1part;               // defer mode: [16][kC1Rep] conv1 wgrad replicas (atomics; zeroed by the forward)
  unsigned* tick;              // [kTicks] arrival counters (zero at rest)
  float* g;                    // flat gradient buffer: the folded (canonical) conv gradients land here
  long long c1w, c1b, c2w, c2b;   // flat offsets of conv1.weight / conv1.bias / conv2.weight / conv2.bias
  // fused fc-bucket all-reduce (W > 1 "fused" schedule): W blocks [0, ar_nvb) run the xGMI peer
  // protocol's virtual blocks over ar_buf once their own work is done
  pde::PeerDev pd;
  float* ar_buf;
  long long ar_n;
  int ar_nvb, ar_two;
  float* c1img;                // ext mode: [B][520] conv1 wgrad|bgrad partial per image (plain stores)
};
// Where the conv weight gradients are reduced (template MODE of k_conv_bwd2):
enum { kBwdFold = 0,    // in-launch: last-arriving W block per k slice folds the 16 slabs (write-through),
                        // conv1 as int64 fixed-point atomics folded by the last D block -> canonical grads
       kBwdDefer = 1,   // W = 1: slabs (plain stores) + float-atomic conv1 replicas in the flat buffer,
                        // folded by the flat optimizer's fold blocks (no reduction seam on the chain)
       kBwdExt = 2 };   // comm path: slabs + per-image conv1 partials, plain stores only; a small
                        // deterministic fold launch (k_conv_grad_fold) writes the canonical gradients
                        // the all-reduce needs

// write-through (sc1) stores and L1-bypassing (sc1) loads for the in-kernel hand-offs
// (MI355X_MICROARCH.md, inter-workgroup visibility: sc1 stores + vmcnt(0) + barrier + one agent-scope
// add; the last adder reads with sc1 loads)
__device__ __forceinline__ void st_wt(float* p, float v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ float ld_wt(const float* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ long long ld_wt64(const long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// One agent-scope arrival add by thread 0 after every wave drained its stores; true in every thread
// of the block whose add completed the count.
__device__ __forceinline__ bool arrive_last(unsigned* ctr, unsigned count, int* flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0)
    *flag = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == count - 1;
  __syncthreads();
  return *flag != 0;
}

struct Bwd2Gather {      // next-batch prefetch (nullptr X: off)
  const float* X;
  const long long* labels;
  const int* idx;
  int n_idx;
  const long long* ctr;  // batch counter, already advanced to the next batch by fc1
  int nbatches;
  int stride;            // batch size of the sampler's batches
  float* Xdst;
  long long* Ydst;
  int* rows_dst;
};

__device__ __forceinline__ void lds_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

template <bool PROF, int MODE>
__global__ __launch_bounds__(512) void k_conv_bwd2(const float* __restrict__ Xb, const float* __restrict__ P1,
                                                   const uint8_t* __restrict__ A1, const float* __restrict__ dP2m,
                                                   const uint8_t* __restrict__ A2, const float* __restrict__ W2c,
                                                   int B, Bwd2Opt op,
                                                   const float* __restrict__ row_loss, const int* __restrict__ row_hit,
                                                   double* __restrict__ loss_sum,
                                                   unsigned long long* __restrict__ correct, Bwd2Gather ga,
                                                   int dbg, unsigned long long* __restrict__ prof) {
  __shared__ __attribute__((aligned(16))) float smem[kBwd2Lds];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, lg = l >> 4;
  PMARK(0);
  const int G = (B + kNIG - 1) / kNIG;             // images per W group (<= 8: B <= 128)
  const int nW = kNIG * 16, nD = 2 * B, npair = min(nW, nD);
  int* lflag = reinterpret_cast<int*>(smem + kL_FLAG);
  const int h = blockIdx.x;
  int role, idx;
  if (h < 2 * npair) {
    role = h & 1;
    idx = h >> 1;
  } else {
    role = nW > nD ? 0 : 1;
    idx = npair + (h - 2 * npair);
  }
  if constexpr (PROF) {
    if (t == 0) prof[(size_t)blockIdx.x * 8 + 7] = role + 1;
  }
  const float4* P1v = reinterpret_cast<const float4*>(P1);
  if ((dbg >> role) & 1) return;     // ablation only (tools/lenet_phases.py --bwd-dbg): 1 = no W, 2 = no D
  if (role == 0) {
    // =============================== role W: conv2 wgrad ===============================
    const int ig = idx >> 4, kp = idx & 15, img0 = ig * G;
    const int ci_base = (32 * kp) / 25;
    const float4* Gv = reinterpret_cast<const float4*>(dP2m);
    const uint4* Av = reinterpret_cast<const uint4*>(A2);
    float4 v4[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int e = t + 512 * j;                  // piece id in [0, 8*358)
      const int ii = min(e / 358, kWImgs - 1), pc = e - (e / 358) * 358;
      const int b = min(img0 + min(ii, G - 1), B - 1);
      const int q = max(pc - 250, 0), ch = min(ci_base + q / 36, 19);
      const float4* src = pc < 200 ? Gv + (size_t)b * 200 + pc
                        : pc < 250 ? reinterpret_cast<const float4*>(Av + (size_t)b * 50 + (pc - 200))
                                   : P1v + (size_t)b * 720 + ch * 36 + (q % 36);
      v4[j] = *src;
    }
    // side jobs: meters (block 0) and the next-batch prefetch chain (its waits come after the MFMAs)
    const bool meter = (idx == 0) && row_loss && loss_sum;
    float mloss = 0.f, mhit = 0.f;
    if (meter && t < B) {
      mloss = row_loss[t];
      mhit = (float)row_hit[t];
    }
    const int grow = idx >> 1, ghalf = idx & 1;
    const bool gjob = ga.X != nullptr && grow < B;
    long long gnb = 0;
    if (gjob) gnb = *ga.ctr;                                                           // link 1
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int e = t + 512 * j;
      if (e < kWImgs * 358) {
        const int ii = e / 358, pc = e - ii * 358;
        float* img = smem + ii * kWImgStride;
        if (pc < 200) {                             // pooled gradient: co = pc / 4, 4 floats
          *reinterpret_cast<float4*>(img + kWG + (pc >> 2) * 20 + 4 * (pc & 3)) = v4[j];
        } else if (pc < 250) {                      // 16 codes of one channel -> 20-byte row
          uint32_t* cd = reinterpret_cast<uint32_t*>(img + kWC) + (pc - 200) * 5;
          cd[0] = __float_as_uint(v4[j].x);
          cd[1] = __float_as_uint(v4[j].y);
          cd[2] = __float_as_uint(v4[j].z);
          cd[3] = __float_as_uint(v4[j].w);
        } else {
          reinterpret_cast<float4*>(img + kWP)[pc - 250] = v4[j];
        }
      }
    }
    if (t < 160) smem[kWImgs * kWImgStride + t] = t < 80 ? 1.f : 0.f;   // B operand of the k >= 500 columns
    if (meter) {
      const float ls = wave_sum(mloss), hs = wave_sum(mhit);
      if (l == 0) {
        smem[kBwd2Lds - 16 + w] = ls;
        smem[kBwd2Lds - 8 + w] = hs;
      }
    }
    int gsrc = 0;
    if (gjob) gsrc = ga.idx[min((gnb % ga.nbatches) * ga.stride + grow, (long long)ga.n_idx - 1)];   // link 2
    lds_barrier();
    PMARK(1);
    if (meter && t == 0) {
      float tl = 0.f, th = 0.f;
      for (int k = 0; k < 8; ++k) {
        tl += smem[kBwd2Lds - 16 + k];
        th += smem[kBwd2Lds - 8 + k];
      }
      loss_sum[0] += (double)tl;
      correct[0] += (unsigned long long)(th + 0.5f);
    }
    const int ct = w & 3, kt = 2 * kp + (w >> 2);
    const int co = ct * 16 + (l & 15), coc = min(co, 49);
    const float com = co < 50 ? 1.f : 0.f;
    const int kk = kt * 16 + (l & 15);
    const int kc = min(kk, 499), ci = kc / 25, rem = kc - ci * 25, kh = rem / 5, kw = rem - kh * 5;
    const int boff = (ci - ci_base) * 144 + (kh + (lg >> 1)) * 12 + kw + 4 * (lg & 1);
    const float* cst = smem + kWImgs * kWImgStride + (kk == 500 ? 0 : 80);   // ones | zeros
    f32x4 acc0 = {0.f}, acc1 = {0.f};
#pragma unroll 2
    for (int ii = 0; ii < kWImgs; ++ii) {
      const float* gi = smem + ii * kWImgStride;
      const uint8_t* ci8 = reinterpret_cast<const uint8_t*>(gi + kWC) + coc * 20 + 2 * (lg & 1);
      const float* gq = gi + kWG + coc * 20 + 2 * (lg & 1);
      const float* p1s = kk < 500 ? gi + kWP + boff : cst;
      const float bm = (ii < G && img0 + ii < B) ? com : 0.f;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const float2 gg = *reinterpret_cast<const float2*>(gq + 4 * c);
        const unsigned short cc = *reinterpret_cast<const unsigned short*>(ci8 + 4 * c);
        const int c0 = cc & 0xff, c1 = cc >> 8, sb = (lg >> 1) * 2;
        const float g0 = gg.x * bm, g1 = gg.y * bm;
        acc0 = mfma16x16x4(c0 == sb ? g0 : 0.f, p1s[24 * c + 0], acc0);
        acc1 = mfma16x16x4(c0 == sb + 1 ? g0 : 0.f, p1s[24 * c + 1], acc1);
        acc0 = mfma16x16x4(c1 == sb ? g1 : 0.f, p1s[24 * c + 2], acc0);
        acc1 = mfma16x16x4(c1 == sb + 1 ? g1 : 0.f, p1s[24 * c + 3], acc1);
      }
    }
    PMARK(2);
    float4 gx = make_float4(0.f, 0.f, 0.f, 0.f);
    if (gjob && t < 98) gx = reinterpret_cast<const float4*>(ga.X + (size_t)gsrc * kImg)[98 * ghalf + t];   // link 3
    // conv2 wgrad partial of image group ig -> slab ig (write-through); no atomics: the last of the 16
    // groups of this k slice folds the slabs in group order, so the gradient is bit-reproducible
    {
      float* sl = op.slab + (size_t)ig * kSlab;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int cor = ct * 16 + lg * 4 + r;
        const float v = acc0[r] + acc1[r];
        if (cor < 50) {
          float* dst = kk < 500 ? sl + cor * 500 + kk : sl + kSlabBias + cor;
          if (kk <= 500) {
            if (MODE != kBwdFold) *dst = v;   // read by the next launch: plain store
            else st_wt(dst, v);               // read by the last-arriving block of this launch: write-through
          }
        }
      }
    }
    if (gjob) {
      if (t < 98) reinterpret_cast<float4*>(ga.Xdst + (size_t)grow * kImg)[98 * ghalf + t] = gx;
      if (ghalf == 0 && t == 0) {
        ga.Ydst[grow] = ga.labels[gsrc];
        ga.rows_dst[grow] = gsrc;
      }
    }
    PMARK(3);
    if constexpr (MODE == kBwdFold) {
    if (arrive_last(op.tick + kp, kNIG, lflag)) {
      PMARK(4);
      // ---- last group of k slice kp: fold the 16 slabs (fixed order) -> canonical gradient ----
      if (t == 0) __hip_atomic_store(op.tick + kp, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __syncthreads();
      // all loads of the fold (4 gradient items x 16 slabs per thread) issued before any use: one
      // dependent round trip, not one per item
      constexpr int kIt = (50 * 32 + 511) / 512;
      float q[kIt][kNIG];
      long long e[kIt];
      int co2[kIt];
#pragma unroll
      for (int u = 0; u < kIt; ++u) {
        const int i = t + 512 * u, co = min(i >> 5, 49), k = min(kp * 32 + (i & 31), 500);
        co2[u] = (i < 50 * 32 && kp * 32 + (i & 31) <= 500) ? co : -1;
        const int so = k < 500 ? co * 500 + k : kSlabBias + co;
#pragma unroll
        for (int r = 0; r < kNIG; ++r) q[u][r] = ld_wt(op.slab + (size_t)r * kSlab + so);
        e[u] = k < 500 ? op.c2w + co * 500 + k : op.c2b + co;
      }
#pragma unroll
      for (int u = 0; u < kIt; ++u) {
        if (co2[u] < 0) continue;
        float gsum = q[u][0];
#pragma unroll
        for (int r = 1; r < kNIG; ++r) gsum += q[u][r];
        op.g[e[u]] = gsum;
      }
    }
    PMARK(5);
    // ---- fused fc-bucket all-reduce across ranks (W > 1 "fused" schedule) ----
    if (op.ar_nvb > 0 && idx < op.ar_nvb)
      pde::peer_ar_f32_vblock(op.pd, op.ar_buf, op.ar_buf, op.ar_n, 1.f, idx, op.ar_nvb, op.ar_two != 0,
                              reinterpret_cast<uint32_t*>(smem + kL_PEER));
    }   // kBwdFold
    PMARK(6);
    return;
  }
  // =============================== role D ===============================
  const int b = idx >> 1, hh = idx & 1;
  float* dys = smem + kD_DY2;
  float* T = smem + kD_T;
  float* p1s = smem + kD_P1;
  uint8_t* c1s = reinterpret_cast<uint8_t*>(smem + kD_C1);
  float* xs = smem + kD_X;
  float* dp1 = smem + kD_DP1;
  // ---- loads: dgrad A operand (both passes), dY2 in gather order, image, P1 / A1 of the half ----
  const int kt = w >> 1, pt = w & 1;
  const int kl = kt * 32 + (l & 31);
  const float km = kl < 125 ? 1.f : 0.f;
  float av[2][25];
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    const float* wa = W2c + (l >> 5) * 500 + (10 * hh + 5 * p) * 25 + min(kl, 124);
#pragma unroll
    for (int s2 = 0; s2 < 25; ++s2) av[p][s2] = wa[2 * s2 * 500];
  }
  // dY2[co][oh][ow] = g[co][pq] if code[co][pq] == sub else 0: thread i reads the pooled value and its
  // code straight from global memory and writes dY2 in address order (conflict-free)
  float gy[7];
  uint8_t gcode[7];
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const int i = min(t + 512 * r, 3199), co = i >> 6, px = i & 63, oh = px >> 3, ow = px & 7;
    const int q = co * 16 + (oh >> 1) * 4 + (ow >> 1);
    gy[r] = dP2m[(size_t)b * kFeat + q];
    gcode[r] = A2[(size_t)b * kFeat + q];
  }
  const float4 xv = reinterpret_cast<const float4*>(Xb + (size_t)b * kImg)[min(t, kImg / 4 - 1)];
  const float4 pv = P1v[(size_t)b * 720 + hh * 360 + min(t, 359)];
  const uint32_t cv = reinterpret_cast<const uint32_t*>(A1 + (size_t)b * kP1 + hh * 1440)[min(t, 359)];
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const int i = t + 512 * r;
    if (i < 3200) {
      const int px = i & 63, sub = ((px >> 3) & 1) * 2 + (px & 1);
      dys[i] = gcode[r] == sub ? gy[r] : 0.f;
    }
  }
  if (t < kImg / 4) reinterpret_cast<float4*>(xs)[t] = xv;
  if (t < 360) {
    reinterpret_cast<float4*>(p1s)[t] = pv;
    reinterpret_cast<uint32_t*>(c1s)[(t / 36) * 37 + (t % 36)] = cv;    // 148-byte code rows
  }
  lds_barrier();
  PMARK(1);
  // ---- two passes of 5 input channels: dgrad T[125 k'][64 px] = W2^T dY2 on v_mfma_f32_32x32x2_f32,
  // then col2im dP1[ci][ih][iw] = sum_{kh,kw} T[ci,kh,kw][ih-kh][iw-kw] ----
#pragma unroll
  for (int p = 0; p < 2; ++p) {
    {
      const float* bp = dys + (l >> 5) * 64 + pt * 32 + (l & 31);
      f32x16 acc = {0.f};
#pragma unroll
      for (int s2 = 0; s2 < 25; ++s2) acc = mfma32x32x2(av[p][s2] * km, bp[2 * s2 * 64], acc);
#pragma unroll
      for (int r = 0; r < 16; ++r)
        T[(kt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 64 + pt * 32 + (l & 31)] = acc[r];
    }
    lds_barrier();
    if (p == 0) PMARK(2);
    // col2im as a gather (fixed summation order) + ReLU mask of P1.  (Measured and rejected: each lane
    // adding its 16 T values into dP1 with LDS atomics straight from the accumulator, no T image and
    // no gather pass -- ds_add_f32 made the step 91 us instead of 55.5, profiles/r3_lenet/.)
    // All 25 taps of an output are read before any is summed, each at ONE per-output base address plus
    // an immediate: tap (kh, kw) of output (ih, iw) is T[25 cl + 5 kh + kw][8 (ih - kh) + (iw - kw)]
    // = base + 312 kh + 63 kw with base = 1600 cl + 8 ih + iw -- an out-of-window tap reads a
    // neighbouring in-bounds T entry (the offset is >= 0 and < 128 x 64) that the sum then drops, in
    // the same (kh, kw) order as the masked form.  (Summing as the reads came made hipcc wait for
    // every ds_read; per-tap clamped addresses cost ~190 VALU per output, this form ~100.)
#pragma unroll
    for (int r = 0; r < 2; ++r) {
      const int o = t + 512 * r;
      if (o < 720) {
        const int cl = o / 144, pos = o - cl * 144, ih = pos / 12, iw = pos - ih * 12;
        const float* tb = T + cl * 1600 + 8 * ih + iw;
        float tv[25];
#pragma unroll
        for (int kh = 0; kh < 5; ++kh)
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) tv[kh * 5 + kw] = tb[312 * kh + 63 * kw];
        const int c = 5 * p + cl;
        const float pm = p1s[c * 144 + pos];
        float sacc = 0.f;
#pragma unroll
        for (int kh = 0; kh < 5; ++kh) {
          const bool rok = ih >= kh && ih < kh + 8;
#pragma unroll
          for (int kw = 0; kw < 5; ++kw) {
            const bool ok = rok && iw >= kw && iw < kw + 8;
            sacc += ok ? tv[kh * 5 + kw] : 0.f;
          }
        }
        dp1[c * 145 + pos] = pm > 0.f ? sacc : 0.f;
      }
    }
    lds_barrier();
    if (p == 0) PMARK(3);
  }
  PMARK(4);
  // ---- conv1 wgrad|bgrad: C[c][tap] = sum_pos dY1[c][pos] * [X(pos + tap) | 1], dY1 unpooled on the fly:
  // pos = 144kq + 4s + lg -> pooled index pq = 36kq + ((4s/24)>>1)*12 + (4s%24)/2 + (lg>>1),
  // window slot sub = ((4s/24)&1)*2 + (lg&1); wave = (tap tile nt, K quarter kq) ----
  float* red = dys;                                           // dY2 is dead: [4][16][36] partials
  {
    const int nt = w & 1, kq = w >> 1;
    const int c = l & 15, cc = min(c, 9);
    const bool cin = c < 10;
    const int tap = nt * 16 + (l & 15);
    const bool tin = tap < 25;
    const float tone = tap == 25 ? 1.f : 0.f;
    const int tc = min(tap, 24), th = tc / 5, tw = tc - th * 5;
    const float* dpp = dp1 + cc * 145 + 36 * kq + (lg >> 1);
    const uint8_t* cdp = c1s + cc * 148 + 36 * kq + (lg >> 1);
    const int lsub = lg & 1;
    const float* xp = xs + (6 * kq + th) * 28 + tw + lg;
    f32x4 acc0 = {0.f}, acc1 = {0.f};
    // operands of 12 k-steps read before their MFMAs (unconditional reads: the gradient is selected by
    // the code afterwards; a conditional read made hipcc branch and wait around every step)
#pragma unroll
    for (int chn = 0; chn < 3; ++chn) {
      uint8_t cv[12];
      float dv[12], xv[12];
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        const int s2 = 12 * chn + q;
        const int rr = (4 * s2) / 24, cq = (4 * s2) % 24;     // pos = 144kq + 4s + lg
        const int qo = (rr >> 1) * 12 + cq / 2;
        cv[q] = cdp[qo];
        dv[q] = dpp[qo];
        xv[q] = xp[rr * 28 + cq];
      }
#pragma unroll
      for (int q = 0; q < 12; ++q) {
        const int s2 = 12 * chn + q;
        const int rr = (4 * s2) / 24, sub = (rr & 1) * 2 + lsub;
        const float a = (cv[q] == sub && cin) ? dv[q] : 0.f;     // one select: code match and channel < 10
        const float bv = tin ? xv[q] : tone;                        // tap < 25: the image; 25: ones; else 0
        if (s2 & 1) acc1 = mfma16x16x4(a, bv, acc1);
        else acc0 = mfma16x16x4(a, bv, acc0);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(kq * 16 + lg * 4 + r) * 36 + nt * 16 + (l & 15)] = acc0[r] + acc1[r];
  }
  lds_barrier();
  PMARK(5);
  if (t < 260) {
    // conv1 wgrad|bgrad partial of this image into replica (b % 16): FOLD -- int64 fixed-point adds
    // (integer addition is associative: bit-identical sums whatever order the blocks arrive in)
    const int c = t / 26, tap = t - c * 26;
    const float v = red[c * 36 + tap] + red[(16 + c) * 36 + tap] + red[(32 + c) * 36 + tap] + red[(48 + c) * 36 + tap];
    const int ch = 10 * hh + c;
    const int slot = tap < 25 ? ch * 25 + tap : 512 + ch;
    if constexpr (MODE == kBwdDefer) {   // float atomics into replica (b % 16), folded by the optimizer
      atomicAdd(op.c1part + (size_t)(b % kC1NRep) * kC1Rep + slot, v);
    } else if constexpr (MODE == kBwdExt) {   // this image's partial, plain store; k_conv_grad_fold sums them
      op.c1img[(size_t)b * kC1Img + hh * 260 + t] = v;
    } else {
      // order-free int64 fixed point (2^-40 quantum).  A non-finite or out-of-range partial (|v| >= 2^22
      // would overflow the 2^62 budget of 16 adders) is not converted: it bumps the flag in unused slot
      // 511 of replica 0 and the folding block then writes NaN -- divergence stays visible.
      if (fabsf(v) < 4194304.f)
        atomicAdd(reinterpret_cast<unsigned long long*>(op.c1rep + (size_t)(b % kC1NRep) * kC1Rep + slot),
                  (unsigned long long)__float2ll_rn(v * kC1Scale));
      else
        atomicAdd(reinterpret_cast<unsigned long long*>(op.c1rep + kC1BadSlot), 1ull);
    }
  }
  if (MODE == kBwdFold && arrive_last(op.tick + kTickD, (unsigned)nD, lflag)) {
    // ---- last D block: fold the 16 replicas (exact) -> canonical conv1 gradient, re-zero ----
    if (t == 0) __hip_atomic_store(op.tick + kTickD, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // items: weight t (t < 500), bias t - 500 (t < 512), bias 12 + t (second slot, t < 8); all loads
    // issued before any use: one dependent round trip
    long long q[2][kC1NRep];
    long long e[2];
    int slot[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int bi = u == 0 ? t - 500 : 12 + min(t, 7);                 // bias index when not a weight
      slot[u] = (u == 0 && t < 500) ? t : 512 + min(bi, 19);
      e[u] = (u == 0 && t < 500) ? op.c1w + t : op.c1b + min(bi, 19);
#pragma unroll
      for (int r = 0; r < kC1NRep; ++r) q[u][r] = ld_wt64(op.c1rep + (size_t)r * kC1Rep + slot[u]);
    }
    const bool bad = ld_wt64(op.c1rep + kC1BadSlot) != 0;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if (u == 1 && t >= 8) break;
      long long acc = 0;
#pragma unroll
      for (int r = 0; r < kC1NRep; ++r) acc += q[u][r];
      const float gsum = (float)((double)acc * kC1InvScale);
      op.g[e[u]] = bad ? __builtin_nanf("") : gsum;
    }
    __syncthreads();
    for (int i = t; i < kC1NRep * kC1Rep; i += 512) op.c1rep[i] = 0;
  }
  PMARK(6);
}

// =================================================================================================
// F3 v2: fc2 (500 -> 10) + log_softmax + cross_entropy(log_softmax) + dlogits + fc2 dgrad + ReLU mask,
// ONE ROW PER 256-THREAD BLOCK (B blocks: 128 CUs at B = 128, against 32 four-row blocks in lenet.hip's
// k_head).  Wave w owns hidden units [128w, 128w + 128): lane l holds n0 = 128w + l and n1 = n0 + 64
// (n1 < 500), so every lane issues its 2 H1 + 20 W2 loads in ONE round trip (22 loads, under the
// vmcnt limit; the four-row kernel needed 88 per lane and waited twice).  The ten class partials are
// reduced across the wave by a TRANSPOSED reduction on VALU lane-exchange ops only (no LDS permutes):
// v_permlane32_swap (10 -> 5 live sums per lane), v_permlane16_swap (5 -> 3), DPP row_mirror (3 -> 2),
// row_half_mirror (2 -> 1), two quad_perm steps -- 13 exchanges instead of 10 x 6 dependent
// ds_bpermute butterflies -- then the four waves' class sums meet in 64 B of LDS.  Same math and
// outputs as k_head (the reference applies cross_entropy to log_softmax output, main.py:89, 147).
// =================================================================================================
__device__ __forceinline__ float xswap_sum32(float a, float b) {   // lanes < 32: a(l)+a(l+32); >= 32: b(l-32)+b(l)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
__device__ __forceinline__ float xswap_sum16(float a, float b) {   // even rows: a(l)+a(l+16); odd: b(l-16)+b(l)
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
template <int CTRL>
__device__ __forceinline__ float dpp(float v) {
  return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(v), CTRL, 0xF, 0xF, true));
}
// Class held (fully reduced, in lanes with (l & 3) == 0) after head_class_reduce; -1 = padding lane.
__device__ __forceinline__ int head_class_of_lane(int l) {
  const int j = ((l >> 3) & 1) * 2 + ((l >> 2) & 1);        // index into the 3 sums of stage 2
  const int y = j + 3 * ((l >> 4) & 1);                     // index into the 5 sums of stage 1
  return (j < 3 && y < 5) ? y + 5 * (l >> 5) : -1;
}
__device__ __forceinline__ float head_class_reduce(const float (&x)[10], int l) {
  float y[6];
#pragma unroll
  for (int k = 0; k < 5; ++k) y[k] = xswap_sum32(x[k], x[k + 5]);
  y[5] = 0.f;
  float z[4];
#pragma unroll
  for (int k = 0; k < 3; ++k) z[k] = xswap_sum16(y[k], y[k + 3]);
  z[3] = 0.f;
  const bool lo8 = (l & 8) == 0, lo4 = (l & 4) == 0;
  float u[2];
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    const float send = lo8 ? z[k + 2] : z[k];
    u[k] = (lo8 ? z[k] : z[k + 2]) + dpp<0x140>(send);                       // row_mirror: i <-> 15 - i
  }
  float v = (lo4 ? u[0] : u[1]) + dpp<0x141>(lo4 ? u[1] : u[0]);              // row_half_mirror: i <-> 7 - i
  v += dpp<0xB1>(v);                                                          // quad_perm(1,0,3,2)
  v += dpp<0x4E>(v);                                                          // quad_perm(2,3,0,1)
  return v;
}

template <bool PROF>
__global__ __launch_bounds__(256) void k_head2(const float* __restrict__ H1, int B, const float* __restrict__ W2,
                                               const float* __restrict__ b2, const long long* __restrict__ labels,
                                               float inv_b, float* __restrict__ logp_out, float* __restrict__ dZ2,
                                               float* __restrict__ dZ1, float* __restrict__ row_loss,
                                               int* __restrict__ row_hit, double* __restrict__ loss_sum,
                                               unsigned long long* __restrict__ correct,
                                               unsigned long long* __restrict__ prof) {
  constexpr int kHid = 500, kCls = 10;
  __shared__ __attribute__((aligned(16))) float part[4][16];
  PMARK(0);
  const int row = blockIdx.x, t = threadIdx.x, l = t & 63, w = t >> 6;
  const int n0 = 128 * w + l, n1 = n0 + 64;                // n0 < 448 + 64 <= 500 always
  const bool v1 = n1 < kHid;
  const int n1c = v1 ? n1 : kHid - 1;
  const float* hrow = H1 + (size_t)row * kHid;
  const float h0 = hrow[n0];
  const float h1r = hrow[n1c];
  float wa[kCls], wb[kCls], bias[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    wa[c] = W2[c * kHid + n0];
    wb[c] = W2[c * kHid + n1c];
  }
#pragma unroll
  for (int c = 0; c < kCls; ++c) bias[c] = b2[c];
  const int y = (int)labels[row];
  // every load above is issued before any use: one round trip (the scheduler would otherwise start
  // the dot products after the first few loads and wait again for each later batch)
  __builtin_amdgcn_sched_barrier(0);
  const float h1 = v1 ? h1r : 0.f;
  float x[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) x[c] = fmaf(h1, wb[c], h0 * wa[c]);
  const float red = head_class_reduce(x, l);
  const int cls = head_class_of_lane(l);
  if ((l & 3) == 0 && cls >= 0) part[w][cls] = red;
  __syncthreads();
  PMARK(2);
  float4 pv[4][3];                                   // 12 broadcast b128 reads, one wait
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int k = 0; k < 3; ++k) pv[q][k] = reinterpret_cast<const float4*>(part[q])[k];
  float z[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    const float* a0 = &pv[0][c >> 2].x;
    const float* a1 = &pv[1][c >> 2].x;
    const float* a2 = &pv[2][c >> 2].x;
    const float* a3 = &pv[3][c >> 2].x;
    z[c] = (a0[c & 3] + a1[c & 3]) + (a2[c & 3] + a3[c & 3]) + bias[c];
  }
  // log_softmax once: the model's log_softmax followed by cross_entropy's is the same function
  // (log_softmax is idempotent: logsumexp(log_softmax(z)) = 0), so CE(log_softmax(z)) = -lp[y] and
  // dlogits = softmax(z) - onehot(y) exactly; p reuses the exponentials of the sum
  float m = z[0];
#pragma unroll
  for (int c = 1; c < kCls; ++c) m = fmaxf(m, z[c]);
  float ez[kCls], se = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    ez[c] = expf(z[c] - m);
    se += ez[c];
  }
  const float lse = logf(se), rse = 1.f / se;
  float lp[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) lp[c] = z[c] - m - lse;
  float m2 = lp[0];
  int pred = 0;
#pragma unroll
  for (int c = 1; c < kCls; ++c) {
    if (lp[c] > m2) { m2 = lp[c]; pred = c; }
  }
  float lpy = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) lpy = (c == y) ? lp[c] : lpy;
  const float loss = -lpy;
  const int hit = pred == y ? 1 : 0;
  if (t == 0) {
    if (row_loss) {
      row_loss[row] = loss;
      row_hit[row] = hit;
    } else if (loss_sum) {
      atomicAdd(loss_sum, (double)loss);
      atomicAdd(correct, (unsigned long long)hit);
    }
  }
  if (logp_out && t < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) v = (c == t) ? lp[c] : v;
    logp_out[(size_t)row * kCls + t] = v;
  }
  if (!dZ1) return;
  float dz[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) dz[c] = (ez[c] * rse - (c == y ? 1.f : 0.f)) * inv_b;
  if (t < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) v = (c == t) ? dz[c] : v;
    dZ2[(size_t)row * kCls + t] = v;
  }
  float s0 = 0.f, s1 = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    s0 = fmaf(dz[c], wa[c], s0);
    s1 = fmaf(dz[c], wb[c], s1);
  }
  float* drow = dZ1 + (size_t)row * kHid;
  drow[n0] = h0 > 0.f ? s0 : 0.f;
  if (v1) drow[n1] = h1 > 0.f ? s1 : 0.f;
  PMARK(1);
}

// Ext-mode fold (the comm path's canonical conv gradients, deterministic: fixed summation order).
// Blocks [0, kFoldC2): conv2 -- thread i of the 25088-float slab image sums the 16 slabs in group
// order (16 loads in flight per thread).  Blocks [kFoldC2, +kFoldC1): conv1 -- 16 outputs per block,
// thread (o = t & 15, part = t >> 4) sums images part, part + 16, ... in order, then the 16 parts are
// added in part order through LDS.
constexpr int kFoldC2 = (kSlab + 255) / 256;        // 98
constexpr int kFoldC1 = (kC1Img + 15) / 16;         // 33
__global__ __launch_bounds__(256) void k_conv_grad_fold(const float* __restrict__ slab, const float* __restrict__ c1img,
                                                        int B, float* __restrict__ g, long long c1w, long long c1b,
                                                        long long c2w, long long c2b) {
  const int t = threadIdx.x;
  if (blockIdx.x < kFoldC2) {
    const int i = blockIdx.x * 256 + t;
    const int ic = min(i, kSlab - 1);
    float q[kNIG];
#pragma unroll
    for (int r = 0; r < kNIG; ++r) q[r] = slab[(size_t)r * kSlab + ic];
    float s = q[0];
#pragma unroll
    for (int r = 1; r < kNIG; ++r) s += q[r];
    if (i < 25000) g[c2w + i] = s;
    else if (i >= kSlabBias && i < kSlabBias + 50) g[c2b + (i - kSlabBias)] = s;
    return;
  }
  __shared__ float red[16][17];
  const int o = (blockIdx.x - kFoldC2) * 16 + (t & 15), part = t >> 4, oc = min(o, kC1Img - 1);
  float s = 0.f;
  constexpr int kMaxPer = 8;                         // B <= 128 images: 8 per part
  float q[kMaxPer];
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k) {
    const int b = part + 16 * k;
    q[k] = c1img[(size_t)min(b, B - 1) * kC1Img + oc];
  }
#pragma unroll
  for (int k = 0; k < kMaxPer; ++k)
    if (part + 16 * k < B) s += q[k];
  red[part][t & 15] = s;
  __syncthreads();
  if (t < 16 && o < kC1Img) {
    float a = red[0][t];
#pragma unroll
    for (int p = 1; p < 16; ++p) a += red[p][t];
    const int hh = o / 260, rem = o - hh * 260, c = rem / 26, tap = rem - c * 26, ch = 10 * hh + c;
    if (tap < 25) g[c1w + ch * 25 + tap] = a;
    else g[c1b + ch] = a;
  }
}

// Ext-mode fold FUSED with the in-place one-shot all-reduce of the whole flat gradient buffer (the
// W > 1 "serial ...:pfold" schedule: one launch where there were two, k_conv_grad_fold + the standalone
// peer_inplace_kernel).  Blocks [0, nfold) are k_conv_grad_fold's fold blocks at 512 threads (the same
// per-output summation order, so the canonical conv gradients are bit-identical), writing with
// system-scope write-through stores, then bumping sync[0].  Blocks [nfold, grid) are virtual blocks
// vb = 0.. of the in-place one-shot over the registered buffer (peer_inplace_kernel's vector map,
// flag slots and per-slot call counting, pde_peer_dev.h): a block whose vectors touch the conv range
// first waits until every fold block is done -- it has a higher block id than every fold block, so
// those are already dispatched and never wait on anything -- and the last such block resets the
// counters for the next launch (graph replays).  The sum is in fixed rank order: replicas stay
// bit-identical.
constexpr int kFoldC2w = (kSlab + 511) / 512;       // 49 conv2 fold blocks of 512
constexpr int kFoldC1w = (kC1Img + 31) / 32;        // 17 conv1 fold blocks (32 outputs x 16 parts)
constexpr int kFoldNw = kFoldC2w + kFoldC1w;

struct FoldArArgs {
  pde::PeerIpDev d;
  const float* slab;
  const float* c1img;
  int B;
  long long c1w, c1b, c2w, c2b;   // element offsets of the conv slots in the registered buffer
  long long n4;                   // 16-byte vectors all-reduced: [0, n4) of the registered buffer
  long long lo4, hi4;             // vectors the fold writes (the conv range)
  unsigned* sync;                 // [0] fold blocks done, [1] waiting blocks past their wait
  int nwait;                      // AR blocks whose vectors touch [lo4, hi4)
  float scale;
};

// one fold block (k_conv_grad_fold's summation order at 512 threads; write-through stores), then its
// arrival on sync[0]
__device__ __forceinline__ void fold_ar_fold_block(const FoldArArgs& a, float (*red)[33]) {
  const int t = threadIdx.x;
  const pde::PeerIpDev& d = a.d;
  const __amdgpu_buffer_rsrc_t ro = pde::ipd_rsrc(d.data[d.rank], d.bytes);
  auto st_sys = [&](long long e, float v) {   // write-through: in memory once drained (peers read it there)
    __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(v), ro, (int)(e * 4), 0, pde::kIpdAuxSys);
  };
  if ((int)blockIdx.x < kFoldC2w) {
    const int i = blockIdx.x * 512 + t;
    const int ic = min(i, kSlab - 1);
    float q[kNIG];
#pragma unroll
    for (int r = 0; r < kNIG; ++r) q[r] = a.slab[(size_t)r * kSlab + ic];
    float sum = q[0];
#pragma unroll
    for (int r = 1; r < kNIG; ++r) sum += q[r];
    if (i < 25000) st_sys(a.c2w + i, sum);
    else if (i >= kSlabBias && i < kSlabBias + 50) st_sys(a.c2b + (i - kSlabBias), sum);
  } else {
    const int o = ((int)blockIdx.x - kFoldC2w) * 32 + (t & 31), part = t >> 5, oc = min(o, kC1Img - 1);
    float sum = 0.f;
    constexpr int kMaxPer = 8;
    float q[kMaxPer];
#pragma unroll
    for (int k = 0; k < kMaxPer; ++k) q[k] = a.c1img[(size_t)min(part + 16 * k, a.B - 1) * kC1Img + oc];
#pragma unroll
    for (int k = 0; k < kMaxPer; ++k)
      if (part + 16 * k < a.B) sum += q[k];
    red[part][t & 31] = sum;
    __syncthreads();
    if (t < 32 && o < kC1Img) {
      float acc = red[0][t];
#pragma unroll
      for (int p = 1; p < 16; ++p) acc += red[p][t];
      const int hh = o / 260, rem = o - hh * 260, c = rem / 26, tap = rem - c * 26, ch = 10 * hh + c;
      if (tap < 25) st_sys(a.c1w + ch * 25 + tap, acc);
      else st_sys(a.c1b + ch, acc);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // every wave's write-through stores acknowledged
  __syncthreads();
  if (t == 0) __hip_atomic_fetch_add(a.sync, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// an all-reduce block that reads conv-range data: wait until every fold block has arrived (their ids are
// lower, so they are all dispatched already and wait on nothing); *s_bad <- 1 on a (never expected) time-out
__device__ __forceinline__ void fold_ar_wait(const FoldArArgs& a, uint32_t* s_bad) {
  if (threadIdx.x == 0) {
    const uint64_t w0 = __builtin_amdgcn_s_memrealtime();
    while (__hip_atomic_load(a.sync, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < (unsigned)kFoldNw) {
      __builtin_amdgcn_s_sleep(1);
      if ((int64_t)(__builtin_amdgcn_s_memrealtime() - w0) > a.d.timeout) { *s_bad = 1u; break; }
    }
  }
  __syncthreads();
}

// the last waiting block resets the counters for the next launch
__device__ __forceinline__ void fold_ar_exit(const FoldArArgs& a) {
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(a.sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    if (prev == (unsigned)a.nwait - 1u) {
      __hip_atomic_store(a.sync + 1, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(a.sync, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

template <int U>
__global__ __launch_bounds__(512) void k_conv_fold_ar(FoldArArgs a) {
  __shared__ float red[16][33];
  __shared__ uint32_t s_call, s_bad;
  const int t = threadIdx.x;
  const pde::PeerIpDev& d = a.d;
  float* own = reinterpret_cast<float*>(d.data[d.rank]);
  if ((int)blockIdx.x < kFoldNw) {
    fold_ar_fold_block(a, red);
    return;
  }
  // ---- in-place one-shot, virtual block vb ----
  const int vb = (int)blockIdx.x - kFoldNw, nvb = (int)gridDim.x - kFoldNw;
  const long long stride = (long long)nvb * 512, t0 = (long long)vb * 512 + t;
  bool waits = false;
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long b0 = (long long)vb * 512 + u * stride;
    waits = waits || (b0 < a.hi4 && b0 + 512 > a.lo4);
  }
  if (t == 0) s_bad = 0u;
  __syncthreads();
  if (waits) fold_ar_wait(a, &s_bad);
  pde::ipd_arrive(d, vb, &s_call);
  if (t == 64 && __hip_atomic_load(d.errc + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) s_bad = 1u;
  __syncthreads();
  const uint32_t target = s_call + 1u;
  const bool failed = s_bad != 0;
  __amdgpu_buffer_rsrc_t rs[pde::kPeerMaxRanks];
#pragma unroll
  for (int p = 0; p < pde::kPeerMaxRanks; ++p) rs[p] = pde::ipd_rsrc(p < d.world ? d.data[p] : d.data[d.rank], d.bytes);
  pde::ipd_barrier<false>(d, 0, vb, target, failed, true, &s_bad);   // A: every rank's buffer holds its input
  pde::peer_vec_t v[U][pde::kPeerMaxRanks];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = t0 + u * stride, ic = i < a.n4 ? i : 0;
#pragma unroll
    for (int p = 0; p < pde::kPeerMaxRanks; ++p)
      if (p < d.world) v[u][p] = pde::ipd_ld(rs[p], ic);
  }
  pde::peer_vec_t res[U];
#pragma unroll
  for (int u = 0; u < U; ++u) res[u] = pde::peer_sum(v[u], d.world, a.scale);   // fixed rank order
  pde::ipd_barrier<true>(d, 1, vb, target, failed, true, &s_bad);    // B: every rank has read every buffer
  const bool bad = s_bad != 0;
  const pde::peer_vec_t nanv = {0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u};
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const long long i = t0 + u * stride;
    if (i < a.n4) reinterpret_cast<pde::peer_vec_t*>(own)[i] = bad ? nanv : res[u];
  }
  if (waits) fold_ar_exit(a);
}

// The two-shot form (W > 2 over real links: each rank reduces one 1/W chunk from every rank, then gathers
// the others' chunks -- 2 (W-1)/W of the buffer over the links instead of W-1 times it).  Every
// all-reduce block waits for the fold (a peer's block reads this rank's conv vectors in any chunk), then
// peer_inplace_kernel's two-shot path: barrier A, reduce-scatter (write-through), barrier B, all-gather,
// barrier C.  R: vectors per thread per iteration (R x W system loads in flight).
template <int R>
__global__ __launch_bounds__(512) void k_conv_fold_ar2(FoldArArgs a) {
  __shared__ float red[16][33];
  __shared__ uint32_t s_call, s_bad;
  const int t = threadIdx.x;
  const pde::PeerIpDev& d = a.d;
  float* own = reinterpret_cast<float*>(d.data[d.rank]);
  if ((int)blockIdx.x < kFoldNw) {
    fold_ar_fold_block(a, red);
    return;
  }
  const int vb = (int)blockIdx.x - kFoldNw, nvb = (int)gridDim.x - kFoldNw;
  const long long stride = (long long)nvb * 512, t0 = (long long)vb * 512 + t;
  if (t == 0) s_bad = 0u;
  __syncthreads();
  fold_ar_wait(a, &s_bad);
  pde::ipd_arrive(d, vb, &s_call);
  if (t == 64 && __hip_atomic_load(d.errc + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) s_bad = 1u;
  __syncthreads();
  const uint32_t target = s_call + 1u;
  const bool failed = s_bad != 0;
  const int W = d.world;
  __amdgpu_buffer_rsrc_t rs[pde::kPeerMaxRanks];
#pragma unroll
  for (int p = 0; p < pde::kPeerMaxRanks; ++p) rs[p] = pde::ipd_rsrc(p < W ? d.data[p] : d.data[d.rank], d.bytes);
  const __amdgpu_buffer_rsrc_t ro = rs[d.rank];
  const long long chunk4 = (a.n4 + W - 1) / W, lo = (long long)d.rank * chunk4;
  const long long len = lo + chunk4 <= a.n4 ? chunk4 : (a.n4 > lo ? a.n4 - lo : 0);
  pde::ipd_barrier<false>(d, 0, vb, target, failed, true, &s_bad);   // A: every rank's buffer holds its input
  const pde::peer_vec_t nanv = {0x7FC00000u, 0x7FC00000u, 0x7FC00000u, 0x7FC00000u};
  for (long long i0 = t0; i0 < len; i0 += R * stride) {           // reduce-scatter: my chunk
    pde::peer_vec_t v[R][pde::kPeerMaxRanks];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long long i = i0 + r * stride;
#pragma unroll
      for (int p = 0; p < pde::kPeerMaxRanks; ++p)
        if (p < W) v[r][p] = pde::ipd_ld(rs[p], lo + (i < len ? i : i0));
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long long i = i0 + r * stride;
      const pde::peer_vec_t o = s_bad ? nanv : pde::peer_sum(v[r], W, a.scale);
      if (i < len) __builtin_amdgcn_raw_buffer_store_b128(o, ro, (int)((lo + i) * 16), 0, pde::kIpdAuxSys);
    }
  }
  pde::ipd_barrier<true>(d, 1, vb, target, failed, true, &s_bad);   // B: every chunk reduced, every input read
  const bool bad = s_bad != 0;
  const long long last = a.n4 - 1;
  for (long long i0 = t0; i0 < chunk4; i0 += R * stride) {        // all-gather: chunk q from its owner q
    pde::peer_vec_t v[R][pde::kPeerMaxRanks];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long long i = i0 + r * stride;
#pragma unroll
      for (int q = 0; q < pde::kPeerMaxRanks; ++q) {
        const long long gq = (long long)q * chunk4 + i;
        if (q < W && q != d.rank) v[r][q] = pde::ipd_ld(rs[q], gq < last ? gq : last);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const long long i = i0 + r * stride;
#pragma unroll
      for (int q = 0; q < pde::kPeerMaxRanks; ++q) {
        const long long gq = (long long)q * chunk4 + i;
        if (q < W && q != d.rank && i < chunk4 && gq <= last)
          reinterpret_cast<pde::peer_vec_t*>(own)[gq] = bad ? nanv : v[r][q];
      }
    }
  }
  pde::ipd_barrier<true>(d, 2, vb, target, failed, true, &s_bad);   // C: every rank has gathered
  fold_ar_exit(a);
}

__global__ void k_pack_w2_v2(const float* __restrict__ w2, float* __restrict__ dst) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e < 25000) dst[pde_lenet_wp_index(e)] = w2[e];
}

}  // namespace

extern "C" {

hipError_t pde_lenet_conv_fwd2(const float* Xb, int B, const float* w1, const float* b1, const float* Wp,
                               const float* b2, float* P1, uint8_t* A1, float* P2, uint8_t* A2, float* zero_ptr,
                               int zero_n, hipStream_t st) {
  unsigned long long* prof = pde_lenet_prof_slot(0);
  // conv1 on the VALU (default) or on 32x32x2 f32 MFMA tiles (PDE_LENET_CONV1=mfma, A/B runs)
  static const int valu = [] {
    const char* e = getenv("PDE_LENET_CONV1");
    return (e != nullptr && e[0] == 'm') ? 0 : 1;
  }();
#define PDE_CF2_LAUNCH(P, V)                                                                                  \
  hipLaunchKernelGGL((k_conv_fwd2<P, V>), dim3(B, 2), dim3(512), 0, st, Xb, w1, b1, Wp, b2, P1, A1, P2, A2, zero_ptr, \
                     zero_n, P ? prof : nullptr)
  if (prof) {
    if (valu) PDE_CF2_LAUNCH(true, true);
    else PDE_CF2_LAUNCH(true, false);
  } else {
    if (valu) PDE_CF2_LAUNCH(false, true);
    else PDE_CF2_LAUNCH(false, false);
  }
#undef PDE_CF2_LAUNCH
  return hipGetLastError();
}

hipError_t pde_lenet_gather(const float* X, const long long* labels, const int* idx, int n_idx, const long long* ctr,
                            int nbatches, int B, float* Xdst, long long* Ydst, int* rows_dst, hipStream_t st) {
  hipLaunchKernelGGL(k_gather, dim3((B + 3) / 4), dim3(256), 0, st, X, labels, idx, n_idx, ctr, nbatches, B, Xdst,
                     Ydst, rows_dst);
  return hipGetLastError();
}

hipError_t pde_lenet_conv_bwd2(const float* Xb, const float* P1, const uint8_t* A1, const float* dP2m,
                               const uint8_t* A2, const float* W2c, int B, const PdeLenetBwdOpt* o,
                               const float* row_loss, const int* row_hit, double* loss_sum, unsigned long long* correct,
                               const float* gX, const long long* glabels, const int* gidx, int gn_idx,
                               const long long* gctr, int gnbatches, int gstride, float* gXdst, long long* gYdst,
                               int* grows, int dbg, hipStream_t st) {
  if (B < 1 || B > 128) return hipErrorInvalidValue;                  // 16 image groups of <= 8 images
  const int nblk = kNIG * 16 + 2 * B;
  Bwd2Gather ga{gX, glabels, gidx, gn_idx, gctr, gnbatches, gstride, gXdst, gYdst, grows};
  Bwd2Opt op{};
  op.slab = o->slab;
  op.c1rep = o->c1rep;
  op.c1part = o->c1part;
  op.tick = o->tick;
  op.g = o->g;
  op.c1w = o->c1w; op.c1b = o->c1b; op.c2w = o->c2w; op.c2b = o->c2b;
  op.c1img = o->c1img;
  const int mode = o->defer == 1 ? kBwdDefer : (o->defer == 2 ? kBwdExt : kBwdFold);
  if (mode == kBwdExt && op.c1img == nullptr) return hipErrorInvalidValue;
  if (o->peer_dev != nullptr && o->ar_buf != nullptr && o->ar_n > 0) {
    std::memcpy(&op.pd, o->peer_dev, sizeof(op.pd));
    op.ar_buf = o->ar_buf;
    op.ar_n = o->ar_n;
    op.ar_two = o->ar_two;
    const long long n4 = o->ar_n / 4, work = o->ar_two ? (n4 + op.pd.world - 1) / op.pd.world : n4;
    op.ar_nvb = (int)std::min<long long>(32, std::max<long long>(1, (work + 511) / 512));
  }
  unsigned long long* prof = pde_lenet_prof_slot(4);
#define PDE_BWD2_LAUNCH(P, F)                                                                                  \
  hipLaunchKernelGGL((k_conv_bwd2<P, F>), dim3(nblk), dim3(512), 0, st, Xb, P1, A1, dP2m, A2, W2c, B, op, row_loss, \
                     row_hit, loss_sum, correct, ga, dbg, P ? prof : nullptr)
  if (prof) {
    if (mode == kBwdDefer) PDE_BWD2_LAUNCH(true, kBwdDefer);
    else if (mode == kBwdExt) PDE_BWD2_LAUNCH(true, kBwdExt);
    else PDE_BWD2_LAUNCH(true, kBwdFold);
  } else {
    if (mode == kBwdDefer) PDE_BWD2_LAUNCH(false, kBwdDefer);
    else if (mode == kBwdExt) PDE_BWD2_LAUNCH(false, kBwdExt);
    else PDE_BWD2_LAUNCH(false, kBwdFold);
  }
#undef PDE_BWD2_LAUNCH
  return hipGetLastError();
}

hipError_t pde_lenet_conv_grad_fold(const float* slab, const float* c1img, int B, float* g, long long c1w, long long c1b,
                                    long long c2w, long long c2b, hipStream_t st) {
  if (B < 1 || B > 128) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_conv_grad_fold, dim3(kFoldC2 + kFoldC1), dim3(256), 0, st, slab, c1img, B, g, c1w, c1b, c2w, c2b);
  return hipGetLastError();
}

hipError_t pde_lenet_conv_fold_ar(const void* ipdev, const float* slab, const float* c1img, int B, long long c1w,
                                 long long c1b, long long c2w, long long c2b, long long n, long long lo, long long hi,
                                 unsigned* sync, float scale, int two, hipStream_t st) {
  if (B < 1 || B > 128 || n <= 0 || (n & 3) || (lo & 3) || (hi & 3) || lo < 0 || hi > n || lo >= hi)
    return hipErrorInvalidValue;
  FoldArArgs a{};
  std::memcpy(&a.d, ipdev, sizeof(a.d));
  if (n * 4 > a.d.bytes || c1w < lo || c1b + 20 > hi || c2w < lo || c2b + 50 > hi) return hipErrorInvalidValue;
  a.slab = slab; a.c1img = c1img; a.B = B;
  a.c1w = c1w; a.c1b = c1b; a.c2w = c2w; a.c2b = c2b;
  a.n4 = n / 4; a.lo4 = lo / 4; a.hi4 = hi / 4;
  a.sync = sync;
  a.scale = scale;
  if (two) {
    // the standalone two-shot's grid: one thread per chunk vector, at most 64 blocks (fewer when ranks
    // share a GPU); R x W system loads in flight per thread
    const int W = a.d.world;
    const long long chunk4 = (a.n4 + W - 1) / W;
    const long long nvb = std::max(1LL, std::min<long long>(std::min(64, a.d.block_cap), (chunk4 + 511) / 512));
    a.nwait = (int)nvb;
    const dim3 grid((unsigned)(kFoldNw + nvb));
    if (W <= 2) hipLaunchKernelGGL(k_conv_fold_ar2<4>, grid, dim3(512), 0, st, a);
    else if (W <= 4) hipLaunchKernelGGL(k_conv_fold_ar2<2>, grid, dim3(512), 0, st, a);
    else hipLaunchKernelGGL(k_conv_fold_ar2<1>, grid, dim3(512), 0, st, a);
    return hipGetLastError();
  }
  // vectors per thread: 2 (the standalone one-shot's measured best), more only to fit the grid cap
  const int cap = std::min(a.d.block_cap, (int)pde::kPeerMaxBlocks);
  int U = 2;
  while (U < 4 && (a.n4 + 512LL * U - 1) / (512LL * U) > cap) U *= 2;
  const long long nvb = (a.n4 + 512LL * U - 1) / (512LL * U);
  if (nvb > cap) return hipErrorInvalidValue;                       // does not fit one-shot: no fused route
  const long long stride = nvb * 512;
  int nwait = 0;
  for (long long vb = 0; vb < nvb; ++vb) {
    bool w = false;
    for (int u = 0; u < U; ++u) {
      const long long b0 = vb * 512 + u * stride;
      w = w || (b0 < a.hi4 && b0 + 512 > a.lo4);
    }
    nwait += w ? 1 : 0;
  }
  a.nwait = nwait;
  const dim3 grid((unsigned)(kFoldNw + nvb));
  if (U == 2) hipLaunchKernelGGL(k_conv_fold_ar<2>, grid, dim3(512), 0, st, a);
  else hipLaunchKernelGGL(k_conv_fold_ar<4>, grid, dim3(512), 0, st, a);
  return hipGetLastError();
}

hipError_t pde_lenet_head2(const float* H1, int B, const float* W2, const float* b2, const long long* labels,
                           float inv_b, float* logp_out, float* dZ2, float* dZ1, float* row_loss, int* row_hit,
                           double* loss_sum, unsigned long long* correct, hipStream_t st) {
  if (B < 1) return hipSuccess;
  unsigned long long* prof = pde_lenet_prof_slot(2);
  if (prof)
    hipLaunchKernelGGL(k_head2<true>, dim3(B), dim3(256), 0, st, H1, B, W2, b2, labels, inv_b, logp_out, dZ2, dZ1,
                       row_loss, row_hit, loss_sum, correct, prof);
  else
    hipLaunchKernelGGL(k_head2<false>, dim3(B), dim3(256), 0, st, H1, B, W2, b2, labels, inv_b, logp_out, dZ2, dZ1,
                       row_loss, row_hit, loss_sum, correct, nullptr);
  return hipGetLastError();
}

hipError_t pde_lenet_pack_w2_v2(const float* w2, float* dst, hipStream_t st) {
  hipLaunchKernelGGL(k_pack_w2_v2, dim3((25000 + 255) / 256), dim3(256), 0, st, w2, dst);
  return hipGetLastError();
}

}  // extern "C"
