// Fused CDNA4 kernels for the reference "toy CNN" (LeNet-style Net of
// /root/reference/mnist/main.py:130-147) trained with Adam + cross-entropy
// (/root/reference/mnist/main.py:78-101).
//
// One training step = 5 launches here (+ the fused Adam of optim.hip):
//   F1 k_conv_fwd : sampler-index gather + conv1(1->20) + bias + ReLU + maxpool (VALU, weights in LDS)
//                   + conv2(20->50) implicit GEMM on v_mfma_f32_32x32x2_f32 + bias + ReLU + maxpool;
//                   conv1's output never leaves LDS on the way to conv2 (it is also stored for backward)
//   F2 k_fc1_fwd  : fc1 (800->500) on v_mfma_f32_16x16x4_f32, split-K over 4 waves + bias + ReLU
//   F3 k_head     : fc2 (500->10) + log_softmax + cross_entropy(log_softmax) + dlogits + fc2-dgrad +
//                   ReLU mask -> dZ1; per-row loss/hit for the device-side meters
//   B1 k_fc_bwd   : dP2 = dZ1 W1 (MFMA, masked by ReLU), dW1|db1 and dW2|db2 (MFMA, bias grads as a
//                   ones column of the B operand), meters folded by one thread (no atomics)
//   B2 k_conv_bwd : conv2 wgrad|bgrad (MFMA, ones column, atomics over 8-image groups) + conv2 dgrad
//                   (MFMA) with col2im as an LDS gather + maxpool1/ReLU backward + conv1 wgrad|bgrad (MFMA)
// Latency rule used throughout (MI355X_MICROARCH.md, cycle constants): a dependent global round
// trip costs ~1 us on data another XCD just wrote, so every kernel issues ALL of its global loads
// into registers first (compile-time-sized, clamped indices, never a branch around a load), waits
// once, and then works from LDS/registers.
// Layouts (fp32 throughout, the reference model is fp32):
//   X    [N][784] dataset (device resident), idx int32 sampler indices, labels int64
//   P1   [B][20][12][12] pooled conv1 out, A1 uint8 argmax code (dy*2+dx) per pooled element
//   P2   [B][800] pooled conv2 out flattened as view(-1, 800) (c*16 + h*4 + w), A2 codes
//   H1   [B][500] relu(fc1)
//   Wt2  [500][64] conv2 weight repacked: row k' = (kh*5+kw)*20+ci, column co (zero for co >= 50)
#include "pde_hip.h"
#include "pde_kernels.h"
#include "pde_peer_dev.h"

#include <algorithm>
#include <cstring>

namespace {

constexpr int kImg = 784;      // 28*28
constexpr int kP1 = 2880;      // 20*12*12
constexpr int kFeat = 800;     // 50*4*4
constexpr int kHid = 500;
constexpr int kCls = 10;

// In-kernel phase timestamps (tools/lenet_phases.py): PROF instantiations record s_memrealtime
// (100 MHz, chip-global) per block at phase boundaries into prof[block * 8 + phase]; slot 7 holds
// the block's role.  Production launches use the PROF = false instantiations (no extra code).
#define PMARK(ph)                                                                             \
  do {                                                                                        \
    if constexpr (PROF) {                                                                     \
      if (threadIdx.x == 0) prof[(size_t)blockIdx.x * 8 + (ph)] = __builtin_amdgcn_s_memrealtime(); \
    }                                                                                         \
  } while (0)
#define PROLE(r)                                                                              \
  do {                                                                                        \
    if constexpr (PROF) {                                                                     \
      if (threadIdx.x == 0) prof[(size_t)blockIdx.x * 8 + 7] = (r);                          \
    }                                                                                         \
  } while (0)

// -------------------------------------------------------------------------------------------------
// Batch bookkeeping: the batch's sample rows either come from an explicit index list, or from an
// epoch permutation indexed by a device-side batch counter (hipGraph replay needs no host work).
struct BatchSrc {
  const int* idx;              // epoch permutation (or per-batch list) or nullptr (identity)
  const long long* step;       // device batch counter or nullptr
  int nbatches;                // batches per epoch when step != nullptr
  int batch;                   // stride between batches in idx
  int n_idx;                   // length of idx (reads are clamped: a full-size launch on a ragged tail is safe)
};

__device__ __forceinline__ int sample_row(const BatchSrc& s, int b) {
  if (!s.idx) return b;
  long long off = 0;
  if (s.step) off = (long long)((*s.step) % s.nbatches) * s.batch;
  return s.idx[min(off + b, (long long)s.n_idx - 1)];
}

// =================================================================================================
// F1: conv1 + conv2 forward.  grid (B, 2 co-tiles), block 256.
// Block (b, ct) stages the ct-th 32 columns of Wt2 (64 KB) and its image; the weight loads are
// issued right after the image / conv1 weights so their latency hides under conv1's compute.
// conv1 (all 20 channels; recomputed by both co-tile blocks, it is 0.29 MFLOP vs conv2's 1.6) runs
// on v_mfma_f32_32x32x2_f32 with the max-pool done on the accumulator registers.
// conv2: wave w = (px-half w&1, K-half w>>1), 125 x v_mfma_f32_32x32x2_f32 on one accumulator
// (dependent latency == issue interval), A = weights from LDS, B = im2col of conv1's LDS output.
// Side jobs: block ct==0 stores P1/A1 (for backward) and the batch's row/label; the grid zeroes
// the atomically-accumulated conv gradient bucket.
// =================================================================================================
template <int KK>
__device__ __forceinline__ f32x16 conv2_mainloop(const float* wa, const float* xb) {
  f32x16 acc = {0.f};
#pragma unroll
  for (int s = 0; s < 125; ++s) {
    const int S = KK * 125 + s;             // MFMA step; k' = 2S + (lane>>5)
    const int grp = S / 10, kh = grp / 5, kw = grp % 5, ci0 = (S % 10) * 2;
    acc = mfma32x32x2(wa[(2 * S) * 32], xb[ci0 * 144 + kh * 12 + kw], acc);
  }
  return acc;
}

constexpr int kFwdWs = 500 * 32;           // staged weight slice (floats)
constexpr int kFwdLds = kFwdWs + kP1 + kImg + 528;

template <bool PROF>
__global__ __launch_bounds__(256) void k_conv_fwd(const float* __restrict__ X, BatchSrc src,
                                                  const long long* __restrict__ labels_all,
                                                  const float* __restrict__ w1, const float* __restrict__ b1,
                                                  const float* __restrict__ Wt2, const float* __restrict__ b2,
                                                  float* __restrict__ P1, uint8_t* __restrict__ A1,
                                                  float* __restrict__ P2, uint8_t* __restrict__ A2,
                                                  int* __restrict__ cur_row, long long* __restrict__ cur_lbl,
                                                  float* __restrict__ zero_ptr, int zero_n, int dbg,
                                                  unsigned long long* __restrict__ prof) {
  PMARK(0);
  // dbg (ablation only): 1 skip conv1 compute, 2 skip conv2 MFMA, 4 skip weight-slice staging,
  // 8 row = b (no counter -> idx -> image load chain), 16 no P1/A1 stores, 32 no bucket zeroing
  __shared__ __attribute__((aligned(16))) float smem[kFwdLds];
  float* ws = smem;                        // [500 k'][32 co]
  float* xs = smem + kFwdWs;               // conv1 output [20][144]
  float* xin = xs + kP1;                   // input image [784]
  float* w1s = xin + kImg;                 // conv1 weight [500] + bias [20] (+pad)
  const int b = blockIdx.x, ct = blockIdx.y, t = threadIdx.x, l = t & 63, w = t >> 6;
  if (zero_ptr && !(dbg & 32)) {
    const int nb = gridDim.x * gridDim.y, bid = ct * gridDim.x + b;
    for (int i = bid * 256 + t; i < zero_n; i += nb * 256) zero_ptr[i] = 0.f;
  }
  const int row = (dbg & 8) ? b : sample_row(src, b);
  PMARK(1);
  // ---- phase 0: issue every global load (image + conv1 weights first, then the weight slice) ----
  const float4 xv = reinterpret_cast<const float4*>(X + (size_t)row * kImg)[min(t, kImg / 4 - 1)];
  const float4 wv = reinterpret_cast<const float4*>(w1)[min(t, 124)];
  const float bv1 = b1[min(t, 19)];
  float4 tmp[16];
  {
    const float4* wsrc = reinterpret_cast<const float4*>(Wt2) + ct * 8;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      const int e = (dbg & 4) ? t : min(t + 256 * i, 3999);   // 4000 float4: row e>>3, column chunk e&7
      tmp[i] = wsrc[(e >> 3) * 16 + (e & 7)];
    }
  }
  if (t < kImg / 4) reinterpret_cast<float4*>(xin)[t] = xv;
  if (t < 125) reinterpret_cast<float4*>(w1s)[t] = wv;
  if (t < 20) w1s[500 + t] = bv1;
  if (ct == 0 && t == 0) {
    if (cur_row) cur_row[b] = row;
    if (cur_lbl && labels_all) cur_lbl[b] = labels_all[row];
  }
  __syncthreads();
  PMARK(2);
  // ---- phase 1: conv1 on v_mfma_f32_32x32x2_f32 + bias + relu + maxpool ----
  // C[m][ch] = sum_tap im2col[m][tap] * W1[ch][tap] with m = 4 * pooled_pos + sub (sub = dy*2+dx):
  // rows (r&3) of the accumulator are the 4 sub-positions of one pooled position, so the 2x2 max
  // pool (first maximum in scan order wins, as ATen) happens in registers.  576 = 18 tiles of 32.
  if (!(dbg & 1)) {
    const int ch = l & 31, hi = l >> 5;
    const float chm = ch < 20 ? 1.f : 0.f;
    float wb[13];
#pragma unroll
    for (int s2 = 0; s2 < 13; ++s2) {
      const int tap = 2 * s2 + hi;
      wb[s2] = (tap < 25) ? w1s[min(ch, 19) * 25 + min(tap, 24)] * chm : 0.f;
    }
    const float bch = w1s[500 + min(ch, 19)];
    for (int tile = w; tile < 18; tile += 4) {
      const int m = tile * 32 + ch, pp = m >> 2, sub = m & 3;
      const float* xa = xin + (2 * (pp / 12) + (sub >> 1)) * 28 + 2 * (pp % 12) + (sub & 1);
      f32x16 acc = {0.f};
#pragma unroll
      for (int s2 = 0; s2 < 13; ++s2) {
        const int t0 = 2 * s2, t1 = min(2 * s2 + 1, 24);
        const int off = hi ? (t1 / 5) * 28 + t1 % 5 : (t0 / 5) * 28 + t0 % 5;
        acc = mfma32x32x2(xa[off], wb[s2], acc);
      }
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
          if (ct == 0 && !(dbg & 16)) {
            const size_t o = (size_t)b * kP1 + ch * 144 + pq;
            P1[o] = best;
            A1[o] = (uint8_t)code;
          }
        }
      }
    }
  }
  PMARK(3);
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (t + 256 * i < 4000) reinterpret_cast<float4*>(ws)[t + 256 * i] = tmp[i];
  __syncthreads();
  PMARK(4);
  // ---- phase 2: conv2 implicit GEMM ----
  const int ph2 = w & 1, kk = w >> 1, khalf = l >> 5, pl = l & 31;
  const float* xb = xs + khalf * 144 + (ph2 * 4 + (pl >> 3)) * 12 + (pl & 7);
  const float* wa = ws + khalf * 32 + pl;
  f32x16 acc = {0.f};
  if (!(dbg & 2)) acc = kk == 0 ? conv2_mainloop<0>(wa, xb) : conv2_mainloop<1>(wa, xb);
  else acc[0] = wa[0] + xb[0];
  PMARK(5);
  __syncthreads();                         // ws is reused as the reduction buffer below
  float* red = smem;                       // [2][32][65]
#pragma unroll
  for (int r = 0; r < 16; ++r)
    red[(kk * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf) * 65 + ph2 * 32 + pl] = acc[r];
  __syncthreads();
  PMARK(6);
  const int nco = ct == 0 ? 32 : 18;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int o = t + 256 * r;
    if (o < nco * 16) {
      const int cl = o >> 4, ph = (o >> 2) & 3, pw = o & 3, co = ct * 32 + cl;
      const float bv = b2[co];
      float best = -1.f; int code = 0;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int p = (2 * ph + (q >> 1)) * 8 + 2 * pw + (q & 1);
        const float v = fmaxf(red[cl * 65 + p] + red[(32 + cl) * 65 + p] + bv, 0.f);
        if (v > best) { best = v; code = q; }
      }
      const size_t oi = (size_t)b * kFeat + co * 16 + ph * 4 + pw;
      P2[oi] = best;
      A2[oi] = (uint8_t)code;
    }
  }
  PMARK(7);
}

// =================================================================================================
// F2: H1 = relu(P2 @ W1^T + b1).  grid (32 n-tiles, ceil(B/16) m-tiles), block 256 (4 waves split K).
// Lane-contiguous K: each lane loads 4 consecutive k of its A row and of its B column (W1 row) as
// one float4; MFMA j uses element j.  The 13 K-chunks of a wave are fully unrolled so all 26
// 16-B loads are in flight before the first MFMA.  Block (0,0) also advances the engine's device
// counters (optimizer step, batch position): F1 of this step has already consumed them and the
// fused Adam that follows reads the new optimizer step.
// =================================================================================================
template <bool PROF>
__global__ __launch_bounds__(256) void k_fc1_fwd(const float* __restrict__ P2, int B, const float* __restrict__ W,
                                                 const float* __restrict__ bias, float* __restrict__ H1,
                                                 long long* __restrict__ ctr, int nctr,
                                                 unsigned long long* __restrict__ prof) {
  PMARK(0);
  __shared__ float red[4][16][17];
  const int nt = blockIdx.x, mt = blockIdx.y, t = threadIdx.x, l = t & 63, w = t >> 6;
  if (ctr && nt == 0 && mt == 0 && t == 0)
    for (int c = 0; c < nctr; ++c) ctr[c] += 1;
  const int row = mt * 16 + (l & 15), n = nt * 16 + (l & 15), kg = l >> 4;
  const float am = row < B ? 1.f : 0.f, bm = n < kHid ? 1.f : 0.f;
  const float4* ap = reinterpret_cast<const float4*>(P2 + (size_t)min(row, B - 1) * kFeat + kg * 4);
  const float4* bp = reinterpret_cast<const float4*>(W + (size_t)min(n, kHid - 1) * kFeat + kg * 4);
  float4 a[13], bb[13];
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const int c = min(w + 4 * i, kFeat / 16 - 1);
    a[i] = ap[c * 4];
    bb[i] = bp[c * 4];
  }
  const float bvv = bias[min(n, kHid - 1)];
  f32x4 acc0 = {0.f}, acc1 = {0.f};
#pragma unroll
  for (int i = 0; i < 13; ++i) {
    const float km = (w + 4 * i < kFeat / 16) ? am : 0.f;
    acc0 = mfma16x16x4(a[i].x * km, bb[i].x * bm, acc0);
    acc1 = mfma16x16x4(a[i].y * km, bb[i].y * bm, acc1);
    acc0 = mfma16x16x4(a[i].z * km, bb[i].z * bm, acc0);
    acc1 = mfma16x16x4(a[i].w * km, bb[i].w * bm, acc1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][(l >> 4) * 4 + r][l & 15] = acc0[r] + acc1[r];
  __syncthreads();
  if (w == 0) {
    // C layout: lane (l&15) owns column n, rows (l>>4)*4 + r
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int i = (l >> 4) * 4 + r, j = l & 15, gm = mt * 16 + i;
      if (gm < B && n < kHid) {
        const float v = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j] + bvv;
        H1[(size_t)gm * kHid + n] = fmaxf(v, 0.f);
      }
    }
  }
  PMARK(1);
}

// =================================================================================================
// F3: fc2 + log_softmax + cross_entropy + backward to dZ1.  grid ceil(B/4), block 256: wave = row.
// The reference computes F.cross_entropy(F.log_softmax(z)) (main.py:89,147): the loss applies a
// second log_softmax to the log-probs.  We evaluate exactly that chain, and its gradient
//   dlogp = (softmax(logp) - onehot)/B ; dz = dlogp - exp(logp) * sum(dlogp)
// then dH1 = dz @ W2, dZ1 = dH1 * (H1 > 0).
// Lane l owns hidden units n = l + 64 j (j < 8): every load/store instruction is 256 contiguous B.
// Meters: per-row loss / hit written to row_loss/row_hit (summed later by one thread of B1, no
// same-address atomics in the hot path); if those are null and loss_sum is given (eval), one
// atomic per block after an LDS reduction.
// Modes: dZ1 == nullptr -> forward/eval only.
// =================================================================================================
template <bool PROF>
__global__ __launch_bounds__(256) void k_head(const float* __restrict__ H1, int B, const float* __restrict__ W2,
                                              const float* __restrict__ b2, const long long* __restrict__ labels,
                                              float inv_b, float* __restrict__ logp_out, float* __restrict__ dZ2,
                                              float* __restrict__ dZ1, float* __restrict__ row_loss,
                                              int* __restrict__ row_hit, double* __restrict__ loss_sum,
                                              unsigned long long* __restrict__ correct,
                                              unsigned long long* __restrict__ prof) {
  PMARK(0);
  __shared__ float sl[4];
  __shared__ int sh[4];
  const int t = threadIdx.x, l = t & 63, wv = t >> 6, row = blockIdx.x * 4 + wv;
  const bool live = row < B;
  const int rc = min(row, B - 1);
  float h[8], w2[kCls][8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = min(l + 64 * j, kHid - 1);
    h[j] = H1[(size_t)rc * kHid + n];
#pragma unroll
    for (int c = 0; c < kCls; ++c) w2[c][j] = W2[c * kHid + n];
  }
  const int y = (int)labels[rc];
  float bias[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) bias[c] = b2[c];
#pragma unroll
  for (int j = 0; j < 8; ++j) h[j] = (l + 64 * j < kHid) ? h[j] : 0.f;
  float z[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) s = fmaf(h[j], w2[c][j], s);
    z[c] = s;
  }
#pragma unroll
  for (int o = 32; o > 0; o >>= 1)
#pragma unroll
    for (int c = 0; c < kCls; ++c) z[c] += __shfl_xor(z[c], o, 64);
#pragma unroll
  for (int c = 0; c < kCls; ++c) z[c] += bias[c];
  // model output: log_softmax(z)
  float m = z[0];
#pragma unroll
  for (int c = 1; c < kCls; ++c) m = fmaxf(m, z[c]);
  float se = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) se += expf(z[c] - m);
  const float lse = logf(se);
  float lp[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) lp[c] = z[c] - m - lse;
  // F.cross_entropy(lp, y) = nll(log_softmax(lp))
  float m2 = lp[0];
  int pred = 0;
#pragma unroll
  for (int c = 1; c < kCls; ++c) {
    if (lp[c] > m2) { m2 = lp[c]; pred = c; }
  }
  float se2 = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) se2 += expf(lp[c] - m2);
  const float lse2 = logf(se2);
  float lpy = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) lpy = (c == y) ? lp[c] - m2 - lse2 : lpy;
  const float loss = -lpy;
  const int hit = pred == y ? 1 : 0;
  if (row_loss) {
    if (live && l == 0) { row_loss[row] = loss; row_hit[row] = hit; }
  } else if (loss_sum) {
    if (l == 0) { sl[wv] = live ? loss : 0.f; sh[wv] = live ? hit : 0; }
    __syncthreads();
    if (t == 0) {
      atomicAdd(loss_sum, (double)(sl[0] + sl[1] + sl[2] + sl[3]));
      atomicAdd(correct, (unsigned long long)(sh[0] + sh[1] + sh[2] + sh[3]));
    }
  }
  if (!live) return;
  if (logp_out && l < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) v = (c == l) ? lp[c] : v;
    logp_out[(size_t)row * kCls + l] = v;
  }
  if (!dZ1) return;
  float dz[kCls], sdl = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    const float dl = (expf(lp[c] - m2 - lse2) - (c == y ? 1.f : 0.f)) * inv_b;
    dz[c] = dl;
    sdl += dl;
  }
#pragma unroll
  for (int c = 0; c < kCls; ++c) dz[c] = dz[c] - expf(lp[c]) * sdl;
  if (l < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) v = (c == l) ? dz[c] : v;
    dZ2[(size_t)row * kCls + l] = v;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) s = fmaf(dz[c], w2[c][j], s);
    const int n = l + 64 * j;
    if (n < kHid) dZ1[(size_t)row * kHid + n] = h[j] > 0.f ? s : 0.f;
  }
  PMARK(1);
}

// F3b (autograd path): backward of log_softmax + fc2 + ReLU from an arbitrary upstream gradient
// g = dL/dlogp (any loss placed after the model):  dz = g - exp(logp) * sum(g); dZ2 = dz;
// dZ1 = (dz @ W2) * (H1 > 0).  grid ceil(B/4), block 256, wave = row.
__global__ __launch_bounds__(256) void k_head_bwd(const float* __restrict__ H1, int B, const float* __restrict__ W2,
                                                  const float* __restrict__ logp, const float* __restrict__ g,
                                                  float* __restrict__ dZ2, float* __restrict__ dZ1) {
  const int t = threadIdx.x, l = t & 63, row = blockIdx.x * 4 + (t >> 6);
  if (row >= B) return;
  float gg[kCls], lpv[kCls], w2[kCls][8], h[8];
#pragma unroll
  for (int c = 0; c < kCls; ++c) { gg[c] = g[(size_t)row * kCls + c]; lpv[c] = logp[(size_t)row * kCls + c]; }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = min(l + 64 * j, kHid - 1);
    h[j] = H1[(size_t)row * kHid + n];
#pragma unroll
    for (int c = 0; c < kCls; ++c) w2[c][j] = W2[c * kHid + n];
  }
  float dz[kCls], sg = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) sg += gg[c];
#pragma unroll
  for (int c = 0; c < kCls; ++c) dz[c] = gg[c] - expf(lpv[c]) * sg;
  if (l < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) v = (c == l) ? dz[c] : v;
    dZ2[(size_t)row * kCls + l] = v;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) s = fmaf(dz[c], w2[c][j], s);
    const int n = l + 64 * j;
    if (n < kHid) dZ1[(size_t)row * kHid + n] = h[j] > 0.f ? s : 0.f;
  }
}

// Block-wide sum of one float per thread (256 threads); every thread gets the result.
__device__ __forceinline__ float block_sum256(float v, float* scratch) {
  v = wave_sum(v);
  if ((threadIdx.x & 63) == 0) scratch[threadIdx.x >> 6] = v;
  __syncthreads();
  const float r = scratch[0] + scratch[1] + scratch[2] + scratch[3];
  __syncthreads();
  return r;
}

// =================================================================================================
// B1: fc backward, three block roles in one launch (all loads of a wave issued before its MFMAs).
//   role C [0, nC)       : dP2m = (dZ1 @ W1) * (P2 > 0)      16x16 tiles, split-K over 4 waves
//   role A [nC, nC+416)  : [dW1 | db1] = dZ1^T @ [P2 | 1]      16x16 tile per wave, K = B; n-tile 50
//                          is the bias tile (B operand = ones column), so db1 costs one MFMA chain
//   role B [.., +8)      : [dW2 | db2] = dZ2^T @ [H1 | 1]      (column 500 of H1 taken as ones)
//                          block 0 also folds F3's per-row loss/hit into the meters (single writer)
// =================================================================================================
constexpr int kBChunk = 128;   // batch rows per unrolled load batch (role A / B)

template <bool PROF>
__global__ __launch_bounds__(256) void k_fc_bwd(const float* __restrict__ P2, const float* __restrict__ H1,
                                                const float* __restrict__ dZ1, const float* __restrict__ dZ2,
                                                const float* __restrict__ W1, int B, float* __restrict__ dP2m,
                                                float* __restrict__ gW1, float* __restrict__ gb1,
                                                float* __restrict__ gW2, float* __restrict__ gb2,
                                                const float* __restrict__ row_loss, const int* __restrict__ row_hit,
                                                double* __restrict__ loss_sum, unsigned long long* __restrict__ correct,
                                                int dbg, int part, unsigned long long* __restrict__ prof) {
  PMARK(0);
  // dbg (ablation only): 1 skip role C, 2 skip role A, 4 skip role B
  // part: 0 = all roles in one launch, 1 = role C only (critical path), 2 = roles A+B only (side stream)
  __shared__ float red[4][16][17];
  __shared__ float scratch[4];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, kg = l >> 4;
  const int mtiles = (B + 15) / 16;
  const int nC = mtiles * 50, nA = 32 * 51;
  // grid order [B | C | A] (part 1: [C], part 2: [B | A]): role B's blocks carry the longest serial
  // chain (K = batch MFMA), so they are dispatched first instead of after the 800+ C/A blocks.
  constexpr int nB = 32;
  const int h = blockIdx.x;
  int role, bid;
  if (part == 1) { role = 1; bid = h; }
  else if (h < nB) { role = 0; bid = h; }
  else if (part == 2) { role = 2; bid = h - nB; }
  else if (h < nB + nC) { role = 1; bid = h - nB; }
  else { role = 2; bid = h - nB - nC; }
  PROLE(role + 1);
  if (role == 1) {
    if (dbg & 1) return;
    // ---- role C: dP2 tile (mt, nt) over K = 500 (hidden); wave w takes K-chunks w, w+4, ... ----
    // XCD-aware order: the mtiles blocks reading one W1 column slab (16 x 500) get consecutive
    // logical ids, i.e. the same XCD and its L2 (nC and the role offsets are multiples of 8).
    const int L = (nC % 8 == 0) ? xcd_remap(bid, nC) : bid;
    const int nt = L / mtiles, mt = L % mtiles;
    const int row = mt * 16 + (l & 15), n = nt * 16 + (l & 15);
    const float am = row < B ? 1.f : 0.f;
    const float* arow = dZ1 + (size_t)min(row, B - 1) * kHid;
    float4 a[8];
    float bv[8][4];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k0 = (w + 4 * i) * 16 + kg * 4, kc = min(k0, kHid - 4);
      a[i] = *reinterpret_cast<const float4*>(arow + kc);
#pragma unroll
      for (int j = 0; j < 4; ++j) bv[i][j] = W1[(size_t)(kc + j) * kFeat + n];
    }
    const float pm = P2[(size_t)min(mt * 16 + (t >> 4), B - 1) * kFeat + nt * 16 + (t & 15)];
    f32x4 acc0 = {0.f}, acc1 = {0.f};
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float km = ((w + 4 * i) * 16 + kg * 4 < kHid) ? am : 0.f;
      acc0 = mfma16x16x4(a[i].x * km, bv[i][0], acc0);
      acc1 = mfma16x16x4(a[i].y * km, bv[i][1], acc1);
      acc0 = mfma16x16x4(a[i].z * km, bv[i][2], acc0);
      acc1 = mfma16x16x4(a[i].w * km, bv[i][3], acc1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][(l >> 4) * 4 + r][l & 15] = acc0[r] + acc1[r];
    __syncthreads();
    const int i = t >> 4, j = t & 15, gm = mt * 16 + i, gn = nt * 16 + j;
    if (gm < B) {
      const float v = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j];
      dP2m[(size_t)gm * kFeat + gn] = pm > 0.f ? v : 0.f;
    }
    PMARK(1);
    return;
  }
  if (role == 2) {
    if (dbg & 2) return;
    // ---- role A: [dW1|db1] tile (mt over 500, nt over 800 + bias tile 50), K = batch ----
    // XCD-aware order: the 32 blocks sharing one P2 column group (B x 64) are consecutive logical
    // ids on one XCD (hardware deals block h to XCD h % 8; nC and nA are multiples of 8).
    // One 16 x 16 tile per block; the 4 waves split K = batch into 32-row slices (8 loads of each
    // operand per lane; a wave streaming all 128 rows made this role a long serial chain), LDS fold.
    const int L = (nC % 8 == 0) ? xcd_remap(bid, nA) : bid;
    const int mt = L % 32, nt = L / 32;                // nt 0..50 (50 = bias tile: ones column)
    const int m = mt * 16 + (l & 15), n = nt * 16 + (l & 15);
    const int mc = min(m, kHid - 1), nc = min(n, kFeat - 1);
    const float mm = m < kHid ? 1.f : 0.f;
    const bool bias_tile = nt == 50;                  // block-uniform
    const float ones = (n == kFeat) ? 1.f : 0.f;
    f32x4 acc0 = {0.f}, acc1 = {0.f};
    for (int b0 = 32 * w; b0 < B; b0 += 128) {
      float av[8], bvv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = b0 + 4 * i + kg, rc = min(r, B - 1);
        av[i] = dZ1[(size_t)rc * kHid + mc] * (r < B ? mm : 0.f);
        bvv[i] = bias_tile ? ones : P2[(size_t)rc * kFeat + nc];
      }
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        acc0 = mfma16x16x4(av[i], bvv[i], acc0);
        acc1 = mfma16x16x4(av[i + 1], bvv[i + 1], acc1);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][(l >> 4) * 4 + r][l & 15] = acc0[r] + acc1[r];
    __syncthreads();
    {
      const int i = t >> 4, j = t & 15, gm = mt * 16 + i, gn = nt * 16 + j;
      const float v = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j];
      if (gm < kHid) {
        if (!bias_tile) __builtin_nontemporal_store(v, gW1 + (size_t)gm * kFeat + gn);   // read by Adam only
        else if (gn == kFeat) gb1[gm] = v;
      }
    }
    PMARK(1);
    return;
  }
  if (dbg & 4) return;
  // ---- role B: [dW2|db2] column tile nt = bid (columns 16nt..16nt+15 over 500 + ones column 500).
  // One block per tile, the 4 waves split K = batch into 32-row slices (8 loads of each operand
  // per lane instead of 64: in-step, one wave streaming the whole batch took ~12 us), LDS fold.
  {
    const int nt = bid;                                // 0..31
    const int n = nt * 16 + (l & 15), nc = min(n, kHid - 1);
    const int c = l & 15, cc = min(c, kCls - 1);
    const float cm = c < kCls ? 1.f : 0.f;
    const float hm = n < kHid ? 1.f : 0.f, ones = n == kHid ? 1.f : 0.f;
    f32x4 acc0 = {0.f}, acc1 = {0.f};
    for (int b0 = 32 * w; b0 < B; b0 += 128) {
      float av[8], bvv[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int r = b0 + 4 * i + kg, rc = min(r, B - 1);
        av[i] = dZ2[(size_t)rc * kCls + cc] * (r < B ? cm : 0.f);
        bvv[i] = H1[(size_t)rc * kHid + nc] * hm + ones;
      }
#pragma unroll
      for (int i = 0; i < 8; i += 2) {
        acc0 = mfma16x16x4(av[i], bvv[i], acc0);
        acc1 = mfma16x16x4(av[i + 1], bvv[i + 1], acc1);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][(l >> 4) * 4 + r][l & 15] = acc0[r] + acc1[r];
    __syncthreads();
    if (t < 160) {                                     // 10 classes x 16 columns
      const int ci = t >> 4, j = t & 15, gn = nt * 16 + j;
      const float v = red[0][ci][j] + red[1][ci][j] + red[2][ci][j] + red[3][ci][j];
      if (gn < kHid) gW2[ci * kHid + gn] = v;
      else if (gn == kHid) gb2[ci] = v;
    }
  }
  if (bid == 0 && row_loss && loss_sum) {
    float ls = 0.f, hs = 0.f;
    for (int r = t; r < B; r += 256) { ls += row_loss[r]; hs += (float)row_hit[r]; }
    const float tl = block_sum256(ls, scratch);
    const float th = block_sum256(hs, scratch);
    if (t == 0) {
      loss_sum[0] += (double)tl;
      correct[0] += (unsigned long long)(th + 0.5f);
    }
  }
  PMARK(1);
}

// =================================================================================================
// B2: conv backward, two block roles in one launch, 512 threads (8 waves) per block.
//   role W [0, nW)       : conv2 wgrad + bias grad.  block = (group of 8 images, 32 k-columns);
//                          wave = (co-tile of 16, k-tile of 16) on v_mfma_f32_16x16x4_f32, K = 8 x 64 px.
//                          The A operand dY2[co][px] is produced on the fly from the pooled gradient and
//                          the argmax codes (no expanded tile), B is the im2col of the P1 slice of the
//                          block's <= 3 input channels; column k = 500 of B is all ones so that column
//                          of the product is the conv2 bias gradient.  Partials are atomically added:
//                          16 adders per address (an earlier 2-image version with 64 adders spent 18 us
//                          in atomics alone, tools/kbench_lenet.py).
//   role D [nW, nW + 4B) : block = (image, group of 5 input channels).
//                          (1) conv2 dgrad T[k][px] = sum_co W[co][k] dY2[co][px] (the group's 125 taps)
//                              on v_mfma_f32_32x32x2_f32, stored to LDS with plain stores;
//                          (2) col2im as a gather (each dP1 element sums its <= 25 taps: no LDS atomics,
//                              which cost 19 us in the scatter-add version), maxpool1 + ReLU mask;
//                          (3) conv1 wgrad|bgrad = dY1[c][576 px] @ [im2col(X) | 1] on
//                              v_mfma_f32_16x16x4_f32 over 4 K-quarters, one atomic per output.
// =================================================================================================
constexpr int kWImgs = 8;                      // images per role-W block
constexpr int kWImgStride = kFeat + 200 + 432; // g800 | codes (800 B) | P1 slice (3 ch x 144)
constexpr int kDysS = 3264;                    // role D carve: dys [50][65] (later dY1 [5][576])
constexpr int kTS = 128 * 65;                  // T [128 k][65]
constexpr int kBwdLds = kDysS + kTS + 720 + kImg + kFeat + 200 + 720 + 180;

template <bool PROF>
__global__ __launch_bounds__(512) void k_conv_bwd(const float* __restrict__ X, const int* __restrict__ rows,
                                                  const float* __restrict__ P1, const uint8_t* __restrict__ A1,
                                                  const float* __restrict__ dP2m, const uint8_t* __restrict__ A2,
                                                  const float* __restrict__ W2c, int B,
                                                  float* __restrict__ gW1c, float* __restrict__ gb1c,
                                                  float* __restrict__ gW2c, float* __restrict__ gb2c,
                                                  int c1_nrep, int c1_rep_stride, const float* __restrict__ row_loss,
                                                  const int* __restrict__ row_hit, double* __restrict__ loss_sum,
                                                  unsigned long long* __restrict__ correct, int dbg,
                                                  pde::PeerDev pd, float* __restrict__ ar_buf, int64_t ar_n,
                                                  int ar_nvb, int ar_two, unsigned long long* __restrict__ prof) {
  PMARK(0);
  // Side blocks (ar_nvb > 0, the W > 1 "fused" schedule): the first ar_nvb blocks after the meters
  // block all-reduce the fc-gradient bucket (complete since fc_bwd) across ranks with the xGMI peer
  // protocol while the other blocks compute the conv gradients -- comm/compute overlap with no
  // extra launch and no cross-stream edge in the graph.
  // conv1 grads go to replica (b % c1_nrep) at a stride of c1_rep_stride floats (the consumer folds
  // the replicas): 128 images adding into 520 addresses was the single largest cost (17 us).
  // dbg (ablation only; 0 in production): 1 skip role W, 2 skip role D, 4 no global atomics,
  // 16 skip conv1 wgrad, 32 skip MFMA loops.  Skipped results stay live.
  __shared__ __attribute__((aligned(16))) float smem[kBwdLds];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, lg = l >> 4;
  const int nIG = (B + kWImgs - 1) / kWImgs, nW = nIG * 16;
  const float4* P1v = reinterpret_cast<const float4*>(P1);
  const float4* Gv = reinterpret_cast<const float4*>(dP2m);
  const uint4* Av = reinterpret_cast<const uint4*>(A2);
  int bid = blockIdx.x;
  if (loss_sum != nullptr) {
    // block 0: fold the head's per-row loss / hit into the device meters.  It rides along this
    // ~20 us kernel (dispatched first) instead of ending fc_bwd's critical chain with two more
    // dependent global round trips (measured: +7 us in-step there).
    if (bid == 0) {
      float ls = 0.f, hs = 0.f;
      for (int r = t; r < B; r += 512) {
        ls += row_loss[r];
        hs += (float)row_hit[r];
      }
      ls = wave_sum(ls);
      hs = wave_sum(hs);
      if (l == 0) {
        smem[w] = ls;
        smem[8 + w] = hs;
      }
      __syncthreads();
      if (t == 0) {
        float tl = 0.f, th = 0.f;
        for (int k = 0; k < 8; ++k) {
          tl += smem[k];
          th += smem[8 + k];
        }
        loss_sum[0] += (double)tl;
        correct[0] += (unsigned long long)(th + 0.5f);
      }
      PROLE(3);
      PMARK(6);
      return;
    }
    bid -= 1;
  }
  if (ar_nvb > 0) {
    if (bid < ar_nvb) {
      pde::peer_ar_f32_vblock(pd, ar_buf, ar_buf, ar_n, 1.f, bid, ar_nvb, ar_two != 0,
                              reinterpret_cast<uint32_t*>(smem));
      return;
    }
    bid -= ar_nvb;
  }
  if (bid < nW) {
    if (dbg & 1) return;
    PROLE(1);
    const int ig = bid >> 4, kp = bid & 15;
    const int ci_base = (32 * kp) / 25;
    // ---- loads for the 8 images: pooled grad (200 float4), codes (50 uint4), P1 slice (108 float4) ----
    // 358 16-B pieces per image, 2864 per block: 6 per thread, all issued before the first LDS store.
    float4 v4[6];
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int e = t + 512 * j;                  // piece id in [0, 8*358)
      const int ii = min(e / 358, kWImgs - 1), pc = e - (e / 358) * 358;
      const int b = min(ig * kWImgs + ii, B - 1);
      const int q = max(pc - 250, 0), ch = min(ci_base + q / 36, 19);
      // one unconditional 16-B load from a selected source (no branch around a load)
      const float4* src = pc < 200 ? Gv + (size_t)b * 200 + pc
                        : pc < 250 ? reinterpret_cast<const float4*>(Av + (size_t)b * 50 + (pc - 200))
                                   : P1v + (size_t)b * 720 + ch * 36 + (q % 36);
      v4[j] = *src;
    }
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int e = t + 512 * j;
      if (e < kWImgs * 358) {
        const int ii = e / 358, pc = e - ii * 358;
        reinterpret_cast<float4*>(smem + ii * kWImgStride)[pc] = v4[j];
      }
    }
    if (t < 160) smem[kWImgs * kWImgStride + t] = t < 80 ? 1.f : 0.f;   // B operand of the k >= 500 columns
    __syncthreads();
    PMARK(1);
    const int ct = w & 3, kt = 2 * kp + (w >> 2);
    const int co = ct * 16 + (l & 15), coc = min(co, 49);
    const float com = co < 50 ? 1.f : 0.f;
    const int kk = kt * 16 + (l & 15);
    const int kc = min(kk, 499), ci = kc / 25, rem = kc - ci * 25, kh = rem / 5, kw = rem - kh * 5;
    // Lane-contiguous pixels: in chunk c (output rows 2c, 2c+1) lane group lg owns row 2c+(lg>>1),
    // columns 4(lg&1)+j, j<4 (MFMA j uses pixel j of the lane's run).  One 8-B read gives the two
    // pooled gradients, one 2-B read their argmax codes, and the P1 reads are immediate offsets.
    const int boff = (ci - ci_base) * 144 + (kh + (lg >> 1)) * 12 + kw + 4 * (lg & 1);
    const float* cst = smem + kWImgs * kWImgStride + (kk == 500 ? 0 : 80);   // ones | zeros
    f32x4 acc0 = {0.f}, acc1 = {0.f};
    if (!(dbg & 32)) {
      for (int ii = 0; ii < kWImgs; ++ii) {
        const float* gi = smem + ii * kWImgStride;
        const uint8_t* ci8 = reinterpret_cast<const uint8_t*>(gi + kFeat) + coc * 16 + 2 * (lg & 1);
        const float* gq = gi + coc * 16 + 2 * (lg & 1);
        const float* p1s = kk < 500 ? gi + kFeat + 200 + boff : cst;
        const float bm = (ig * kWImgs + ii < B) ? com : 0.f;
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
    }
    PMARK(2);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int cor = ct * 16 + lg * 4 + r;
      const float v = acc0[r] + acc1[r];
      if (cor < 50 && (!(dbg & 4) || v == 1234.5f)) {
        if (kk < 500) atomicAdd(&gW2c[cor * 500 + kk], v);
        else if (kk == 500) atomicAdd(&gb2c[cor], v);
      }
    }
    PMARK(6);
    return;
  }
  bid -= nW;
  if (dbg & 2) return;
  PROLE(2);
  // ---- role D ----
  const int b = bid >> 2, cg = bid & 3;
  if (b >= B) return;
  float* dys = smem;                   // [50][65]; later dY1 [5][576]
  float* T = smem + kDysS;             // [128][65]
  float* dp1 = T + kTS;                // [5][144]
  float* xs = dp1 + 720;               // [784]
  float* g800 = xs + kImg;             // [800]
  uint8_t* a800 = reinterpret_cast<uint8_t*>(g800 + kFeat);   // [800]
  float* p1m = g800 + kFeat + 200;     // [720] P1 values of the group's channels
  uint8_t* cds = reinterpret_cast<uint8_t*>(p1m + 720);       // [720] A1 codes
  // ---- loads: dgrad A operand (W2c), dP2m, A2, X row, P1 / A1 of the channel group ----
  const int dmt = w >> 1, dpt = w & 1;                        // dgrad tile: k-tile, px-tile
  const int kl = dmt * 32 + (l & 31);
  const float km = kl < 125 ? 1.f : 0.f;
  const float* wa = W2c + (l >> 5) * 500 + cg * 125 + min(kl, 124);
  float av[25];
#pragma unroll
  for (int s = 0; s < 25; ++s) av[s] = wa[2 * s * 500];
  const float4 gv = Gv[(size_t)b * 200 + min(t, 199)];
  const uint4 a2v = Av[(size_t)b * 50 + min(t, 49)];
  const float4 xv = reinterpret_cast<const float4*>(X + (size_t)rows[b] * kImg)[min(t, kImg / 4 - 1)];
  const float4 pv = P1v[(size_t)b * 720 + cg * 180 + min(t, 179)];
  const uint4 cv = reinterpret_cast<const uint4*>(A1 + (size_t)b * kP1 + cg * 720)[min(t, 44)];
  if (t < 200) reinterpret_cast<float4*>(g800)[t] = gv;
  if (t < 50) reinterpret_cast<uint4*>(a800)[t] = a2v;
  if (t < kImg / 4) reinterpret_cast<float4*>(xs)[t] = xv;
  if (t < 180) reinterpret_cast<float4*>(p1m)[t] = pv;
  if (t < 45) reinterpret_cast<uint4*>(cds)[t] = cv;
  __syncthreads();
  PMARK(1);
  // (0) dY2[co][px] from the pooled gradient + codes
#pragma unroll
  for (int r = 0; r < 7; ++r) {
    const int i = t + 512 * r;
    if (i < 50 * 64) {
      const int c = i >> 6, px = i & 63, oh = px >> 3, ow = px & 7;
      const int q = c * 16 + (oh >> 1) * 4 + (ow >> 1);
      dys[c * 65 + px] = (a800[q] == (oh & 1) * 2 + (ow & 1)) ? g800[q] : 0.f;
    }
  }
  __syncthreads();
  PMARK(2);
  // (1) dgrad tile (dmt, dpt): 25 x 32x32x2 over co = 50
  {
    const float* bp = dys + (l >> 5) * 65 + dpt * 32 + (l & 31);
    f32x16 acc = {0.f};
#pragma unroll
    for (int s = 0; s < 25; ++s) {
      if (dbg & 32) { acc[0] += av[s]; continue; }
      acc = mfma32x32x2(av[s] * km, bp[2 * s * 65], acc);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r)
      T[(dmt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5)) * 65 + dpt * 32 + (l & 31)] = acc[r];
  }
  __syncthreads();
  PMARK(3);
  // (2) col2im gather + maxpool1/relu mask: dP1[cl][ih][iw] = sum_{kh,kw} T[cl*25+kh*5+kw][(ih-kh)*8+iw-kw]
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int o = t + 512 * r;
    if (o < 720) {
      const int cl = o / 144, p = o - cl * 144, ih = p / 12, iw = p - ih * 12;
      float sacc = 0.f;
#pragma unroll
      for (int kh = 0; kh < 5; ++kh) {
        const int oh = ih - kh;
#pragma unroll
        for (int kw = 0; kw < 5; ++kw) {
          const int ow = iw - kw;
          const bool ok = oh >= 0 && oh < 8 && ow >= 0 && ow < 8;
          const int idx = ok ? (cl * 25 + kh * 5 + kw) * 65 + oh * 8 + ow : 0;
          const float tv = T[idx];
          sacc += ok ? tv : 0.f;
        }
      }
      dp1[o] = p1m[o] > 0.f ? sacc : 0.f;
    }
  }
  __syncthreads();
  PMARK(4);
  // (3) dense dY1 [5][576] (into the dead dys region) from dP1 + maxpool1 codes
  float* dy1 = dys;
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int o = t + 512 * r;
    if (o < 720) {
      const int cl = o / 144, p = o - cl * 144, ph = p / 12, pw = p - ph * 12;
      const float g = dp1[o];
      const int code = cds[o];
#pragma unroll
      for (int q = 0; q < 4; ++q)
        dy1[cl * 576 + (2 * ph + (q >> 1)) * 24 + 2 * pw + (q & 1)] = (code == q) ? g : 0.f;
    }
  }
  __syncthreads();
  PMARK(5);
  if (dbg & 16) return;
  // (4) conv1 wgrad|bgrad: C[c][tap] = sum_pos dY1[c][pos] * [X(pos+tap) | 1]; wave = (tap-tile, K-quarter)
  float* red = T;                                             // T is dead: [4][16][33] partials
  {
    const int nt = w & 1, kq = w >> 1;
    const int c = l & 15, cc = min(c, 4);
    const float cmask = c < 5 ? 1.f : 0.f;
    const int tap = nt * 16 + (l & 15);
    const float tmask = tap < 25 ? 1.f : 0.f, tone = tap == 25 ? 1.f : 0.f;
    const int tc = min(tap, 24), th = tc / 5, tw = tc - th * 5;
    const float* ap = dy1 + cc * 576 + kq * 144 + lg;
    const float* xp = xs + (6 * kq + th) * 28 + tw + lg;
    f32x4 acc0 = {0.f}, acc1 = {0.f};
#pragma unroll
    for (int s = 0; s < 36; ++s) {
      const int ohs = (4 * s) / 24, ows = (4 * s) % 24;       // pos = 144kq + 4s + lg
      const float a = ap[4 * s] * cmask;
      const float bv = xp[ohs * 28 + ows] * tmask + tone;
      if (s & 1) acc1 = mfma16x16x4(a, bv, acc1);
      else acc0 = mfma16x16x4(a, bv, acc0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[(kq * 16 + lg * 4 + r) * 33 + nt * 16 + (l & 15)] = acc0[r] + acc1[r];
  }
  __syncthreads();
  if (t < 130) {
    const int c = t / 26, tap = t - c * 26;
    const float v = red[c * 33 + tap] + red[(16 + c) * 33 + tap] + red[(32 + c) * 33 + tap] +
                    red[(48 + c) * 33 + tap];
    if (!(dbg & 4) || v == 1234.5f) {
      const int ch = cg * 5 + c;
      const size_t rep = (size_t)(b % c1_nrep) * c1_rep_stride;
      if (tap < 25) atomicAdd(&gW1c[rep + ch * 25 + tap], v);
      else atomicAdd(&gb1c[rep + ch], v);
    }
  }
  PMARK(6);
}

}  // namespace

// =================================================================================================
// Host launchers (extern "C": no torch headers in device TUs)
// =================================================================================================
namespace {
unsigned long long* g_prof = nullptr;   // host-side switch: non-null -> PROF instantiations
constexpr size_t kProfKernelStride = 4096 * 8;
unsigned long long* prof_slot(int kid) { return g_prof ? g_prof + (size_t)kid * kProfKernelStride : nullptr; }
}  // namespace

extern "C" {

// Phase profiling of the LeNet kernels (tools/lenet_phases.py).  buf: [kernels][4096 blocks][8] u64,
// kernel slots 0 conv_fwd, 1 fc1_fwd, 2 head, 3 fc_bwd, 4 conv_bwd, 5 adam; nullptr switches it off.
void pde_lenet_set_prof(unsigned long long* buf) { g_prof = buf; }
unsigned long long* pde_lenet_prof_slot(int kid) { return prof_slot(kid); }

hipError_t pde_lenet_conv_fwd(const float* X, const int* idx, int n_idx, const long long* step, int nbatches,
                              int stride, const long long* labels_all, int B, const float* w1, const float* b1,
                              const float* Wt2, const float* b2, float* P1, uint8_t* A1, float* P2, uint8_t* A2,
                              int* cur_row, long long* cur_lbl, float* zero_ptr, int zero_n, int dbg, hipStream_t st) {
  BatchSrc src{idx, step, nbatches, stride > 0 ? stride : B, n_idx};
  if (g_prof)
    hipLaunchKernelGGL(k_conv_fwd<true>, dim3(B, 2), dim3(256), 0, st, X, src, labels_all, w1, b1, Wt2, b2, P1, A1, P2,
                       A2, cur_row, cur_lbl, zero_ptr, zero_n, dbg, prof_slot(0));
  else
    hipLaunchKernelGGL(k_conv_fwd<false>, dim3(B, 2), dim3(256), 0, st, X, src, labels_all, w1, b1, Wt2, b2, P1, A1,
                       P2, A2, cur_row, cur_lbl, zero_ptr, zero_n, dbg, nullptr);
  return hipGetLastError();
}

hipError_t pde_lenet_fc1_fwd(const float* P2, int B, const float* W, const float* bias, float* H1, long long* ctr,
                             int nctr, hipStream_t st) {
  if (g_prof)
    hipLaunchKernelGGL(k_fc1_fwd<true>, dim3(32, (B + 15) / 16), dim3(256), 0, st, P2, B, W, bias, H1, ctr, nctr,
                       prof_slot(1));
  else
    hipLaunchKernelGGL(k_fc1_fwd<false>, dim3(32, (B + 15) / 16), dim3(256), 0, st, P2, B, W, bias, H1, ctr, nctr,
                       nullptr);
  return hipGetLastError();
}

hipError_t pde_lenet_head(const float* H1, int B, const float* W2, const float* b2, const long long* labels,
                          float inv_b, float* logp_out, float* dZ2, float* dZ1, float* row_loss, int* row_hit,
                          double* loss_sum, unsigned long long* correct, hipStream_t st) {
  // default: the one-row-per-block kernel of lenet_v2.hip; PDE_LENET_HEAD=1 keeps this file's
  // four-rows-per-block k_head (A/B runs)
  static const bool v1_head = [] {
    const char* e = getenv("PDE_LENET_HEAD");
    return e != nullptr && e[0] == '1';
  }();
  if (!v1_head)
    return pde_lenet_head2(H1, B, W2, b2, labels, inv_b, logp_out, dZ2, dZ1, row_loss, row_hit, loss_sum, correct, st);
  if (g_prof)
    hipLaunchKernelGGL(k_head<true>, dim3((B + 3) / 4), dim3(256), 0, st, H1, B, W2, b2, labels, inv_b, logp_out, dZ2,
                       dZ1, row_loss, row_hit, loss_sum, correct, prof_slot(2));
  else
    hipLaunchKernelGGL(k_head<false>, dim3((B + 3) / 4), dim3(256), 0, st, H1, B, W2, b2, labels, inv_b, logp_out,
                       dZ2, dZ1, row_loss, row_hit, loss_sum, correct, nullptr);
  return hipGetLastError();
}

hipError_t pde_lenet_head_bwd(const float* H1, int B, const float* W2, const float* logp, const float* g, float* dZ2,
                              float* dZ1, hipStream_t st) {
  hipLaunchKernelGGL(k_head_bwd, dim3((B + 3) / 4), dim3(256), 0, st, H1, B, W2, logp, g, dZ2, dZ1);
  return hipGetLastError();
}

hipError_t pde_lenet_fc_bwd(const float* P2, const float* H1, const float* dZ1, const float* dZ2, const float* W1,
                            int B, float* dP2m, float* gW1, float* gb1, float* gW2, float* gb2, const float* row_loss,
                            const int* row_hit, double* loss_sum, unsigned long long* correct, int dbg, int part,
                            hipStream_t st) {
  const int nC = ((B + 15) / 16) * 50, nAB = 32 * 51 + 32;
  const int nblk = part == 1 ? nC : (part == 2 ? nAB : nC + nAB);
  if (g_prof)
    hipLaunchKernelGGL(k_fc_bwd<true>, dim3(nblk), dim3(256), 0, st, P2, H1, dZ1, dZ2, W1, B, dP2m, gW1, gb1, gW2, gb2,
                       row_loss, row_hit, loss_sum, correct, dbg, part, prof_slot(3));
  else
    hipLaunchKernelGGL(k_fc_bwd<false>, dim3(nblk), dim3(256), 0, st, P2, H1, dZ1, dZ2, W1, B, dP2m, gW1, gb1, gW2,
                       gb2, row_loss, row_hit, loss_sum, correct, dbg, part, nullptr);
  return hipGetLastError();
}

hipError_t pde_lenet_conv_bwd(const float* X, const int* rows, const float* P1, const uint8_t* A1,
                              const float* dP2m, const uint8_t* A2, const float* W2c, int B, float* gW1c,
                              float* gb1c, float* gW2c, float* gb2c, int c1_nrep, int c1_rep_stride,
                              const float* row_loss, const int* row_hit, double* loss_sum,
                              unsigned long long* correct, int dbg, const void* peer_dev, float* ar_buf,
                              int64_t ar_n, int ar_two, hipStream_t st) {
  const int meters = (loss_sum && correct && row_loss && row_hit) ? 1 : 0;
  pde::PeerDev pd{};
  int ar_nvb = 0;
  if (peer_dev != nullptr && ar_buf != nullptr && ar_n > 0) {
    std::memcpy(&pd, peer_dev, sizeof(pd));
    const int64_t n4 = ar_n / 4, work = ar_two ? (n4 + pd.world - 1) / pd.world : n4;
    ar_nvb = (int)std::min<int64_t>(64, std::max<int64_t>(1, (work + 511) / 512));
  }
  const int nblk = ((B + kWImgs - 1) / kWImgs) * 16 + 4 * B + meters + ar_nvb;
  if (g_prof)
    hipLaunchKernelGGL(k_conv_bwd<true>, dim3(nblk), dim3(512), 0, st, X, rows, P1, A1, dP2m, A2, W2c, B, gW1c, gb1c,
                       gW2c, gb2c, c1_nrep < 1 ? 1 : c1_nrep, c1_rep_stride, meters ? row_loss : nullptr,
                       meters ? row_hit : nullptr, meters ? loss_sum : nullptr, meters ? correct : nullptr, dbg, pd,
                       ar_buf, ar_n, ar_nvb, ar_two, prof_slot(4));
  else
    hipLaunchKernelGGL(k_conv_bwd<false>, dim3(nblk), dim3(512), 0, st, X, rows, P1, A1, dP2m, A2, W2c, B, gW1c,
                       gb1c, gW2c, gb2c, c1_nrep < 1 ? 1 : c1_nrep, c1_rep_stride, meters ? row_loss : nullptr,
                       meters ? row_hit : nullptr, meters ? loss_sum : nullptr, meters ? correct : nullptr, dbg, pd,
                       ar_buf, ar_n, ar_nvb, ar_two, nullptr);
  return hipGetLastError();
}

}  // extern "C"
