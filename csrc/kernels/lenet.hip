// Fused CDNA4 kernels for the reference "toy CNN" (LeNet-style Net of
// /root/reference/mnist/main.py:130-147) trained with Adam + cross-entropy
// (/root/reference/mnist/main.py:78-101).
//
// One training step = 6 launches (+ the fused Adam of adam.hip):
//   F1 k_conv1_fwd : sampler-index gather + conv1(1->20,5x5) + bias + ReLU + maxpool2x2 (+argmax codes)
//                    + zeroes the atomically-accumulated conv grads (side job)
//   F2 k_conv2_fwd : conv2(20->50,5x5) as implicit GEMM on v_mfma_f32_32x32x2_f32 + bias + ReLU + pool
//   F3 k_fc1_fwd   : fc1 (800->500) on v_mfma_f32_16x16x4_f32, split-K over 4 waves + bias + ReLU
//   F4 k_head      : fc2 (500->10) + log_softmax + cross_entropy(log_softmax) + dlogits + fc2-dgrad +
//                    ReLU mask -> dZ1, device-side loss/accuracy meters (no .item() per step)
//   B1 k_fc_bwd    : dW1/db1 (MFMA), dW2/db2 (VALU), dP2 = dZ1*W1 (MFMA) masked by ReLU
//   B2 k_conv_bwd  : conv2 wgrad (MFMA, atomics over image groups) + conv2 dgrad (MFMA) with col2im in
//                    LDS + maxpool1/ReLU backward + conv1 wgrad (sparse, 1 of 4 pool positions)
// Layout conventions (fp32 throughout, the reference model is fp32):
//   X    [N][784] dataset (device resident), idx int32 sampler indices, labels int64
//   P1   [B][20][12][12] pooled conv1 out, A1 uint8 argmax code (dy*2+dx) per pooled element
//   P2   [B][800] pooled conv2 out flattened as view(-1, 800) (c*16 + h*4 + w), A2 codes
//   H1   [B][500] relu(fc1)
//   Wt2  [500][64] conv2 weight repacked: row k' = (kh*5+kw)*20+ci, column co (zero for co >= 50)
#include "pde_hip.h"
#include "pde_kernels.h"

namespace {

constexpr int kImg = 784;      // 28*28
constexpr int kP1 = 2880;      // 20*12*12
constexpr int kFeat = 800;     // 50*4*4
constexpr int kHid = 500;
constexpr int kCls = 10;

// -------------------------------------------------------------------------------------------------
// Batch bookkeeping shared by the kernels: the batch's sample rows either come from an explicit
// index list, or from an epoch permutation indexed by a device-side step counter (graph replay).
struct BatchSrc {
  const int* idx;              // epoch permutation (or per-batch list) or nullptr (identity)
  const long long* step;       // device step counter or nullptr
  int nbatches;                // batches per epoch when step != nullptr
  int batch;                   // B (stride between batches in idx)
};

__device__ __forceinline__ int sample_row(const BatchSrc& s, int b) {
  if (!s.idx) return b;
  long long off = 0;
  if (s.step) off = (long long)((*s.step) % s.nbatches) * s.batch;
  return s.idx[off + b];
}

// =================================================================================================
// F1: conv1 + bias + relu + maxpool.  grid (B, 4 channel groups of 5), block 192 (3 waves).
// Thread t < 144 owns pooled position (ph, pw) = (t/12, t%12) for the block's 5 channels: a 6x6
// input patch in registers, weights wave-uniform (scalar loads), 500 FMAs.
// =================================================================================================
__global__ __launch_bounds__(192) void k_conv1_fwd(const float* __restrict__ X, BatchSrc src,
                                                   const long long* __restrict__ labels_all,
                                                   const float* __restrict__ w, const float* __restrict__ bias,
                                                   float* __restrict__ P1, uint8_t* __restrict__ A1,
                                                   int* __restrict__ cur_row, long long* __restrict__ cur_lbl,
                                                   float* __restrict__ zero_ptr, int zero_n) {
  const int b = blockIdx.x, g = blockIdx.y, t = threadIdx.x;
  if (zero_ptr) {
    const int nb = gridDim.x * gridDim.y, bid = g * gridDim.x + b;
    for (int i = bid * 192 + t; i < zero_n; i += nb * 192) zero_ptr[i] = 0.f;
  }
  __shared__ __attribute__((aligned(16))) float xs[kImg];
  const int row = sample_row(src, b);
  if (g == 0 && t == 0) {
    if (cur_row) cur_row[b] = row;
    if (cur_lbl && labels_all) cur_lbl[b] = labels_all[row];
  }
  const float4* xsrc = reinterpret_cast<const float4*>(X + (size_t)row * kImg);
  for (int i = t; i < kImg / 4; i += 192) reinterpret_cast<float4*>(xs)[i] = xsrc[i];
  __syncthreads();
  if (t >= 144) return;
  const int ph = t / 12, pw = t - ph * 12;
  float patch[36];
#pragma unroll
  for (int i = 0; i < 6; ++i)
#pragma unroll
    for (int j = 0; j < 6; ++j) patch[i * 6 + j] = xs[(2 * ph + i) * 28 + 2 * pw + j];
#pragma unroll
  for (int c = 0; c < 5; ++c) {
    const int cc = g * 5 + c;
    const float bv = bias[cc];
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
#pragma unroll
    for (int kh = 0; kh < 5; ++kh)
#pragma unroll
      for (int kw = 0; kw < 5; ++kw) {
        const float wv = w[cc * 25 + kh * 5 + kw];
        a0 = fmaf(wv, patch[kh * 6 + kw], a0);
        a1 = fmaf(wv, patch[kh * 6 + kw + 1], a1);
        a2 = fmaf(wv, patch[(kh + 1) * 6 + kw], a2);
        a3 = fmaf(wv, patch[(kh + 1) * 6 + kw + 1], a3);
      }
    // relu then maxpool (first maximum in scan order wins, as ATen's max_pool2d)
    float r0 = fmaxf(a0 + bv, 0.f), r1 = fmaxf(a1 + bv, 0.f), r2 = fmaxf(a2 + bv, 0.f), r3 = fmaxf(a3 + bv, 0.f);
    float best = r0; int code = 0;
    if (r1 > best) { best = r1; code = 1; }
    if (r2 > best) { best = r2; code = 2; }
    if (r3 > best) { best = r3; code = 3; }
    const size_t o = ((size_t)(b * 20 + cc) * 12 + ph) * 12 + pw;
    P1[o] = best;
    A1[o] = (uint8_t)code;
  }
}

// =================================================================================================
// F2: conv2 implicit GEMM.  grid (B, 2 row-halves), block 256.
// Per block: C[co 64][px 32] = sum_{k'<500} Wt2[k'][co] * im2col[k'][px], px = output rows 4h..4h+3.
// wave w: co-tile (w&1), K-half (w>>1), 125 x v_mfma_f32_32x32x2_f32 on one accumulator (the
// instruction's dependent latency equals its issue interval, so one chain runs at full rate).
// A (weights) streams from L2 straight to VGPRs (coalesced 2 x 128 B per step); B from LDS.
// =================================================================================================
template <int KK>
__device__ __forceinline__ f32x16 conv2_mainloop(const float* __restrict__ wa, const float* xb) {
  f32x16 acc = {0.f};
#pragma unroll
  for (int s = 0; s < 125; ++s) {
    const int S = KK * 125 + s;             // MFMA step; k' = 2S + (lane>>5)
    const int grp = S / 10, kh = grp / 5, kw = grp % 5, ci0 = (S % 10) * 2;
    const float a = wa[(2 * S) * 64];
    const float bv = xb[ci0 * 96 + kh * 12 + kw];
    acc = mfma32x32x2(a, bv, acc);
  }
  return acc;
}

__global__ __launch_bounds__(256) void k_conv2_fwd(const float* __restrict__ P1, const float* __restrict__ Wt2,
                                                   const float* __restrict__ bias, float* __restrict__ P2,
                                                   uint8_t* __restrict__ A2) {
  __shared__ __attribute__((aligned(16))) float xs[20 * 96];
  __shared__ float red[2][64][33];
  const int b = blockIdx.x, h = blockIdx.y, t = threadIdx.x, l = t & 63, w = t >> 6;
  const float* src = P1 + (size_t)b * kP1 + 48 * h;
  for (int i = t; i < 20 * 96; i += 256) {
    const int ci = i / 96, r = i - ci * 96;
    xs[i] = src[ci * 144 + r];
  }
  __syncthreads();
  const int ct = w & 1, kk = w >> 1, khalf = l >> 5, px = l & 31;
  const float* xb = xs + khalf * 96 + (px >> 3) * 12 + (px & 7);
  const float* wa = Wt2 + khalf * 64 + ct * 32 + (l & 31);
  f32x16 acc = kk == 0 ? conv2_mainloop<0>(wa, xb) : conv2_mainloop<1>(wa, xb);
#pragma unroll
  for (int r = 0; r < 16; ++r) red[kk][ct * 32 + (r & 3) + 8 * (r >> 2) + 4 * khalf][px] = acc[r];
  __syncthreads();
  for (int o = t; o < 400; o += 256) {
    const int co = o >> 3, ph = (o >> 2) & 1, pw = o & 3;
    const float bv = bias[co];
    float best = -1.f; int code = 0;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int p = (2 * ph + (q >> 1)) * 8 + 2 * pw + (q & 1);
      const float v = fmaxf(red[0][co][p] + red[1][co][p] + bv, 0.f);
      if (v > best) { best = v; code = q; }
    }
    const size_t oi = (size_t)b * kFeat + co * 16 + (2 * h + ph) * 4 + pw;
    P2[oi] = best;
    A2[oi] = (uint8_t)code;
  }
}

// =================================================================================================
// F3: H1 = relu(P2 @ W1^T + b1).  grid (32 n-tiles, ceil(B/16) m-tiles), block 256 (4 waves split K).
// Lane-contiguous K: each lane loads 4 consecutive k of its A row and of its B column (W1 row) as
// one float4; MFMA j uses element j.  Two accumulators hide the 40-cycle dependent latency.
// =================================================================================================
__global__ __launch_bounds__(256) void k_fc1_fwd(const float* __restrict__ P2, int B, const float* __restrict__ W,
                                                 const float* __restrict__ bias, float* __restrict__ H1) {
  __shared__ float red[4][16][17];
  const int nt = blockIdx.x, mt = blockIdx.y, t = threadIdx.x, l = t & 63, w = t >> 6;
  const int row = mt * 16 + (l & 15), n = nt * 16 + (l & 15), kg = l >> 4;
  const float am = row < B ? 1.f : 0.f, bm = n < kHid ? 1.f : 0.f;
  const float4* ap = reinterpret_cast<const float4*>(P2 + (size_t)min(row, B - 1) * kFeat + kg * 4);
  const float4* bp = reinterpret_cast<const float4*>(W + (size_t)min(n, kHid - 1) * kFeat + kg * 4);
  f32x4 acc0 = {0.f}, acc1 = {0.f};
  for (int c = w; c < kFeat / 16; c += 4) {
    const float4 a = ap[c * 4], bb = bp[c * 4];
    acc0 = mfma16x16x4(a.x * am, bb.x * bm, acc0);
    acc1 = mfma16x16x4(a.y * am, bb.y * bm, acc1);
    acc0 = mfma16x16x4(a.z * am, bb.z * bm, acc0);
    acc1 = mfma16x16x4(a.w * am, bb.w * bm, acc1);
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) red[w][(l >> 4) * 4 + r][l & 15] = acc0[r] + acc1[r];
  __syncthreads();
  const int i = t >> 4, j = t & 15, gm = mt * 16 + i, gn = nt * 16 + j;
  if (gm < B && gn < kHid) {
    const float v = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j] + bias[gn];
    H1[(size_t)gm * kHid + gn] = fmaxf(v, 0.f);
  }
}

// =================================================================================================
// F4: fc2 + log_softmax + cross_entropy + backward to dZ1.  grid ceil(B/4), block 256: wave = row.
// The reference computes F.cross_entropy(F.log_softmax(z)) (main.py:89,147): the loss applies a
// second log_softmax to the log-probs.  We evaluate exactly that chain, and its gradient
//   dlogp = (softmax(logp) - onehot)/B ; dz = dlogp - exp(logp) * sum(dlogp)
// then dH1 = dz @ W2, dZ1 = dH1 * (H1 > 0).
// Modes: dZ1 == nullptr -> forward/eval only (loss + accuracy meters, optional logp output).
// =================================================================================================
__global__ __launch_bounds__(256) void k_head(const float* __restrict__ H1, int B, const float* __restrict__ W2,
                                              const float* __restrict__ b2, const long long* __restrict__ labels,
                                              float inv_b, float* __restrict__ logp_out, float* __restrict__ dZ2,
                                              float* __restrict__ dZ1, double* __restrict__ loss_sum,
                                              unsigned long long* __restrict__ correct) {
  const int t = threadIdx.x, l = t & 63, row = blockIdx.x * 4 + (t >> 6);
  if (row >= B) return;
  const int n0 = l * 8;
  float h[8];
  {
    const float4* hp = reinterpret_cast<const float4*>(H1 + (size_t)row * kHid + min(n0, kHid - 4));
    float4 u = hp[0], v = n0 + 4 < kHid ? hp[1] : make_float4(0.f, 0.f, 0.f, 0.f);
    const bool ok = n0 < kHid;
    h[0] = ok ? u.x : 0.f; h[1] = ok ? u.y : 0.f; h[2] = ok ? u.z : 0.f; h[3] = ok ? u.w : 0.f;
    h[4] = v.x; h[5] = v.y; h[6] = v.z; h[7] = v.w;
  }
  float z[kCls];
#pragma unroll
  for (int c = 0; c < kCls; ++c) {
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int n = n0 + j;
      s = fmaf(h[j], n < kHid ? W2[c * kHid + n] : 0.f, s);
    }
    z[c] = wave_sum(s) + b2[c];
  }
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
  const int y = (int)labels[row];
  float lpy = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) lpy = (c == y) ? lp[c] - m2 - lse2 : lpy;
  if (l == 0) {
    if (loss_sum) atomicAdd(loss_sum, (double)(-lpy));
    if (correct && pred == y) atomicAdd(correct, 1ULL);
  }
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
  float o[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = min(n0 + j, kHid - 1);
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) s = fmaf(dz[c], W2[c * kHid + n], s);
    o[j] = h[j] > 0.f ? s : 0.f;
  }
  if (n0 < kHid) {
    float4* dp = reinterpret_cast<float4*>(dZ1 + (size_t)row * kHid + n0);
    dp[0] = make_float4(o[0], o[1], o[2], o[3]);
    if (n0 + 4 < kHid) dp[1] = make_float4(o[4], o[5], o[6], o[7]);
  }
}

// F4b (autograd path): backward of log_softmax + fc2 + ReLU from an arbitrary upstream gradient
// g = dL/dlogp (any loss placed after the model):  dz = g - exp(logp) * sum(g); dZ2 = dz;
// dZ1 = (dz @ W2) * (H1 > 0).  grid ceil(B/4), block 256, wave = row.
__global__ __launch_bounds__(256) void k_head_bwd(const float* __restrict__ H1, int B, const float* __restrict__ W2,
                                                  const float* __restrict__ logp, const float* __restrict__ g,
                                                  float* __restrict__ dZ2, float* __restrict__ dZ1) {
  const int t = threadIdx.x, l = t & 63, row = blockIdx.x * 4 + (t >> 6);
  if (row >= B) return;
  float dz[kCls], sg = 0.f;
#pragma unroll
  for (int c = 0; c < kCls; ++c) sg += g[(size_t)row * kCls + c];
#pragma unroll
  for (int c = 0; c < kCls; ++c) dz[c] = g[(size_t)row * kCls + c] - expf(logp[(size_t)row * kCls + c]) * sg;
  if (l < kCls) {
    float v = 0.f;
#pragma unroll
    for (int c = 0; c < kCls; ++c) v = (c == l) ? dz[c] : v;
    dZ2[(size_t)row * kCls + l] = v;
  }
  const int n0 = l * 8;
  if (n0 >= kHid) return;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const int n = n0 + j;
    if (n < kHid) {
      float s = 0.f;
#pragma unroll
      for (int c = 0; c < kCls; ++c) s = fmaf(dz[c], W2[c * kHid + n], s);
      dZ1[(size_t)row * kHid + n] = H1[(size_t)row * kHid + n] > 0.f ? s : 0.f;
    }
  }
}

// =================================================================================================
// B1: fc backward, three block roles in one launch.
//   role C [0, nC)        : dP2m = (dZ1 @ W1) * (P2 > 0)      16x16 tiles, split-K 4 waves
//   role A [nC, nC+nA)    : dW1 = dZ1^T @ P2                  16x16 tile per wave, K = B
//   role B [.., +8)       : dW2 = dZ2^T @ H1, db1 = sum dZ1, db2 = sum dZ2   (VALU)
// =================================================================================================
__global__ __launch_bounds__(256) void k_fc_bwd(const float* __restrict__ P2, const float* __restrict__ H1,
                                                const float* __restrict__ dZ1, const float* __restrict__ dZ2,
                                                const float* __restrict__ W1, int B, float* __restrict__ dP2m,
                                                float* __restrict__ gW1, float* __restrict__ gb1,
                                                float* __restrict__ gW2, float* __restrict__ gb2) {
  __shared__ float red[4][16][17];
  __shared__ float redB[4][11][64];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int mtiles = (B + 15) / 16;
  const int nC = mtiles * 50, nA = 32 * 13;
  int bid = blockIdx.x;
  if (bid < nC) {
    // ---- role C: dP2 tile (mt, nt) over K = 500 (hidden) ----
    const int mt = bid / 50, nt = bid % 50;
    const int row = mt * 16 + (l & 15), n = nt * 16 + (l & 15), kg = l >> 4;
    const float am = row < B ? 1.f : 0.f;
    const float* ap = dZ1 + (size_t)min(row, B - 1) * kHid + kg * 4;
    f32x4 acc0 = {0.f}, acc1 = {0.f};
    for (int c = w; c < 32; c += 4) {        // chunk c: k in [16c, 16c+16), k < 500
      const int k0 = c * 16 + kg * 4;
      float4 a = k0 < kHid ? *reinterpret_cast<const float4*>(ap + c * 16) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float* bcol = W1 + (size_t)min(k0, kHid - 4) * kFeat + n;
      const float km = k0 < kHid ? 1.f : 0.f;
      acc0 = mfma16x16x4(a.x * am, bcol[0] * km, acc0);
      acc1 = mfma16x16x4(a.y * am, bcol[kFeat] * km, acc1);
      acc0 = mfma16x16x4(a.z * am, bcol[2 * kFeat] * km, acc0);
      acc1 = mfma16x16x4(a.w * am, bcol[3 * kFeat] * km, acc1);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) red[w][(l >> 4) * 4 + r][l & 15] = acc0[r] + acc1[r];
    __syncthreads();
    const int i = t >> 4, j = t & 15, gm = mt * 16 + i, gn = nt * 16 + j;
    if (gm < B) {
      const size_t o = (size_t)gm * kFeat + gn;
      const float v = red[0][i][j] + red[1][i][j] + red[2][i][j] + red[3][i][j];
      dP2m[o] = P2[o] > 0.f ? v : 0.f;
    }
    return;
  }
  bid -= nC;
  if (bid < nA) {
    // ---- role A: dW1 tile (mt over 500, nt over 800), K = batch ----
    const int mt = bid / 13, nt = (bid % 13) * 4 + w;
    if (nt >= 50) return;
    const int m = mt * 16 + (l & 15), n = nt * 16 + (l & 15), kg = l >> 4;
    const int mc = min(m, kHid - 1);
    const float mm = m < kHid ? 1.f : 0.f;
    f32x4 acc0 = {0.f}, acc1 = {0.f};
    int b0 = 0;
    for (; b0 + 8 <= B; b0 += 8) {
      const int r0 = b0 + kg, r1 = b0 + 4 + kg;
      acc0 = mfma16x16x4(dZ1[(size_t)r0 * kHid + mc] * mm, P2[(size_t)r0 * kFeat + n], acc0);
      acc1 = mfma16x16x4(dZ1[(size_t)r1 * kHid + mc] * mm, P2[(size_t)r1 * kFeat + n], acc1);
    }
    for (; b0 < B; b0 += 4) {
      const int r = b0 + kg;
      const float km = r < B ? mm : 0.f;
      const int rc = min(r, B - 1);
      acc0 = mfma16x16x4(dZ1[(size_t)rc * kHid + mc] * km, P2[(size_t)rc * kFeat + n], acc0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int gm = mt * 16 + (l >> 4) * 4 + r;
      if (gm < kHid) gW1[(size_t)gm * kFeat + n] = acc0[r] + acc1[r];
    }
    return;
  }
  bid -= nA;
  // ---- role B: columns n = bid*64 + lane ----
  const int n = bid * 64 + l, nc = min(n, kHid - 1);
  float acc[11];
#pragma unroll
  for (int c = 0; c < 11; ++c) acc[c] = 0.f;
  for (int b = w; b < B; b += 4) {
    const float hv = H1[(size_t)b * kHid + nc];
#pragma unroll
    for (int c = 0; c < kCls; ++c) acc[c] = fmaf(dZ2[b * kCls + c], hv, acc[c]);
    acc[10] += dZ1[(size_t)b * kHid + nc];
  }
#pragma unroll
  for (int c = 0; c < 11; ++c) redB[w][c][l] = acc[c];
  __syncthreads();
  if (w == 0 && n < kHid) {
#pragma unroll
    for (int c = 0; c < kCls; ++c)
      gW2[c * kHid + n] = redB[0][c][l] + redB[1][c][l] + redB[2][c][l] + redB[3][c][l];
    gb1[n] = redB[0][10][l] + redB[1][10][l] + redB[2][10][l] + redB[3][10][l];
  }
  if (bid == 0 && t < kCls) {
    float s = 0.f;
    for (int b = 0; b < B; ++b) s += dZ2[b * kCls + t];
    gb2[t] = s;
  }
}

// Expand the pooled/masked gradient dP2m[b] (+ argmax codes) into dY2 [co][px] in LDS (stride 65).
__device__ __forceinline__ void expand_dy2(float* dys, const float* __restrict__ dP2m, const uint8_t* __restrict__ A2,
                                           int b, int t, int nthreads) {
  const float* g = dP2m + (size_t)b * kFeat;
  const uint8_t* a = A2 + (size_t)b * kFeat;
  for (int i = t; i < 50 * 64; i += nthreads) {
    const int co = i >> 6, px = i & 63, oh = px >> 3, ow = px & 7;
    const int q = co * 16 + (oh >> 1) * 4 + (ow >> 1);
    const int code = (oh & 1) * 2 + (ow & 1);
    dys[co * 65 + px] = (a[q] == code) ? g[q] : 0.f;
  }
}

// =================================================================================================
// B2: conv backward, two block roles in one launch.
//   role W [0, nW)        : conv2 wgrad.  block = (group of 4 images, 4 of the 32 tiles of the
//                           [co 64][k 512] output); wave = one 32x32 tile, K = 64 px per image on
//                           v_mfma_f32_32x32x2_f32; partial sums atomically added to gW2c.
//   role D [nW, nW + 4B)  : block = (image, group of 5 input channels).  conv2 dgrad as the GEMM
//                           T[k][px] = sum_co W[co][k] dY2[co][px] (k restricted to the group's 125
//                           taps), col2im scatter-add into LDS, then maxpool1 + ReLU backward and
//                           conv1 wgrad/bgrad on the 1-of-4 nonzero positions; plus conv2 bias grad.
// =================================================================================================
constexpr int kWImgs = 4;

__global__ __launch_bounds__(256) void k_conv_bwd(const float* __restrict__ X, const int* __restrict__ rows,
                                                  const float* __restrict__ P1, const uint8_t* __restrict__ A1,
                                                  const float* __restrict__ dP2m, const uint8_t* __restrict__ A2,
                                                  const float* __restrict__ W2c, int B,
                                                  float* __restrict__ gW1c, float* __restrict__ gb1c,
                                                  float* __restrict__ gW2c, float* __restrict__ gb2c) {
  __shared__ __attribute__((aligned(16))) float smem[64 * 65 + kP1 + 16];
  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int nIG = (B + kWImgs - 1) / kWImgs, nW = nIG * 8;
  int bid = blockIdx.x;
  if (bid < nW) {
    float* dys = smem;                 // [64][65]
    float* p1s = smem + 64 * 65;       // [20][144]
    const int ig = bid >> 3, tg = bid & 7;
    const int tile = tg * 4 + w, mt = tile >> 4, nt = tile & 15;
    for (int i = 50 * 65 + t; i < 64 * 65; i += 256) dys[i] = 0.f;
    const int kidx = nt * 32 + (l & 31);
    const float kmask = kidx < 500 ? 1.f : 0.f;
    const int kc = min(kidx, 499);
    const int ci = kc / 25, rem = kc - ci * 25, kh = rem / 5, kw = rem - kh * 5;
    const float* bsrc = p1s + ci * 144 + kh * 12 + kw + (l >> 5);
    const float* asrc = dys + (mt * 32 + (l & 31)) * 65 + (l >> 5);
    f32x16 acc = {0.f};
    for (int ii = 0; ii < kWImgs; ++ii) {
      const int b = ig * kWImgs + ii;
      if (b >= B) break;
      __syncthreads();
      expand_dy2(dys, dP2m, A2, b, t, 256);
      const float4* s4 = reinterpret_cast<const float4*>(P1 + (size_t)b * kP1);
      for (int i = t; i < kP1 / 4; i += 256) reinterpret_cast<float4*>(p1s)[i] = s4[i];
      __syncthreads();
#pragma unroll
      for (int s = 0; s < 32; ++s) {
        const float av = asrc[2 * s];
        const float bv = bsrc[(s >> 2) * 12 + 2 * (s & 3)] * kmask;
        acc = mfma32x32x2(av, bv, acc);
      }
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int co = mt * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      if (co < 50 && kidx < 500) atomicAdd(&gW2c[co * 500 + kidx], acc[r]);
    }
    return;
  }
  bid -= nW;
  // ---- role D ----
  const int b = bid >> 2, cg = bid & 3;
  if (b >= B) return;
  float* dys = smem;                   // [50][65] (region rounded to 3264 floats: 16-B aligned carve)
  float* dp1 = smem + 3264;            // [5][144]
  float* xs = dp1 + 720;               // [784]
  uint8_t* cds = reinterpret_cast<uint8_t*>(xs + kImg);  // [720] codes
  for (int i = t; i < 720; i += 256) dp1[i] = 0.f;
  expand_dy2(dys, dP2m, A2, b, t, 256);
  {
    const float4* s4 = reinterpret_cast<const float4*>(X + (size_t)rows[b] * kImg);
    for (int i = t; i < kImg / 4; i += 256) reinterpret_cast<float4*>(xs)[i] = s4[i];
  }
  if (cg == 0 && t < 50) {
    const float* g = dP2m + (size_t)b * kFeat + t * 16;
    float s = 0.f;
#pragma unroll
    for (int p = 0; p < 16; ++p) s += g[p];
    atomicAdd(&gb2c[t], s);
  }
  __syncthreads();
  {
    // wave w: k-tile mt = w (k_local in [32w, 32w+32), valid < 125), both px tiles.
    const int kl = w * 32 + (l & 31);
    const float km = kl < 125 ? 1.f : 0.f;
    const float* wa = W2c + (l >> 5) * 500 + cg * 125 + min(kl, 124);
    const float* b0p = dys + (l >> 5) * 65 + (l & 31);
    f32x16 acc0 = {0.f}, acc1 = {0.f};
#pragma unroll
    for (int s = 0; s < 25; ++s) {
      const float a = wa[2 * s * 500] * km;
      acc0 = mfma32x32x2(a, b0p[2 * s * 65], acc0);
      acc1 = mfma32x32x2(a, b0p[2 * s * 65 + 32], acc1);
    }
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int k = w * 32 + (r & 3) + 8 * (r >> 2) + 4 * (l >> 5);
      if (k < 125) {
        const int cl = k / 25, rem = k - cl * 25, kh = rem / 5, kw = rem - kh * 5;
        const int px0 = l & 31, oh0 = px0 >> 3, ow = px0 & 7;
        atomicAdd(&dp1[cl * 144 + (oh0 + kh) * 12 + ow + kw], acc0[r]);
        atomicAdd(&dp1[cl * 144 + (oh0 + 4 + kh) * 12 + ow + kw], acc1[r]);
      }
    }
  }
  __syncthreads();
  // maxpool1 + relu backward mask, codes to LDS
  for (int i = t; i < 720; i += 256) {
    const size_t gi = (size_t)b * kP1 + cg * 720 + i;
    if (!(P1[gi] > 0.f)) dp1[i] = 0.f;
    cds[i] = A1[gi];
  }
  __syncthreads();
  // conv1 wgrad: 125 outputs (cl, kh, kw) x 2 halves of the 144 pooled positions
  if (t < 250) {
    const int o = t >> 1, half = t & 1;
    const int cl = o / 25, rem = o - cl * 25, kh = rem / 5, kw = rem - kh * 5;
    float s = 0.f, sb = 0.f;
    for (int p = half * 72; p < half * 72 + 72; ++p) {
      const float g = dp1[cl * 144 + p];
      const int code = cds[cl * 144 + p];
      const int ph = p / 12, pw = p - ph * 12;
      const int y = 2 * ph + (code >> 1) + kh, x = 2 * pw + (code & 1) + kw;
      s = fmaf(g, xs[y * 28 + x], s);
      sb += g;
    }
    s += __shfl_xor(s, 1, 64);
    sb += __shfl_xor(sb, 1, 64);
    if (half == 0) {
      const int c = cg * 5 + cl;
      atomicAdd(&gW1c[c * 25 + rem], s);
      if (rem == 0) atomicAdd(&gb1c[c], sb);
    }
  }
}

}  // namespace

// =================================================================================================
// Host launchers (extern "C": no torch headers in device TUs)
// =================================================================================================
extern "C" {

hipError_t pde_lenet_conv1_fwd(const float* X, const int* idx, const long long* step, int nbatches, int stride,
                               const long long* labels_all, int B, const float* w, const float* bias, float* P1,
                               uint8_t* A1, int* cur_row, long long* cur_lbl, float* zero_ptr, int zero_n,
                               hipStream_t st) {
  BatchSrc src{idx, step, nbatches, stride > 0 ? stride : B};
  hipLaunchKernelGGL(k_conv1_fwd, dim3(B, 4), dim3(192), 0, st, X, src, labels_all, w, bias, P1, A1, cur_row,
                     cur_lbl, zero_ptr, zero_n);
  return hipGetLastError();
}

hipError_t pde_lenet_conv2_fwd(const float* P1, int B, const float* Wt2, const float* bias, float* P2, uint8_t* A2,
                               hipStream_t st) {
  hipLaunchKernelGGL(k_conv2_fwd, dim3(B, 2), dim3(256), 0, st, P1, Wt2, bias, P2, A2);
  return hipGetLastError();
}

hipError_t pde_lenet_fc1_fwd(const float* P2, int B, const float* W, const float* bias, float* H1, hipStream_t st) {
  hipLaunchKernelGGL(k_fc1_fwd, dim3(32, (B + 15) / 16), dim3(256), 0, st, P2, B, W, bias, H1);
  return hipGetLastError();
}

hipError_t pde_lenet_head(const float* H1, int B, const float* W2, const float* b2, const long long* labels,
                          float inv_b, float* logp_out, float* dZ2, float* dZ1, double* loss_sum,
                          unsigned long long* correct, hipStream_t st) {
  hipLaunchKernelGGL(k_head, dim3((B + 3) / 4), dim3(256), 0, st, H1, B, W2, b2, labels, inv_b, logp_out, dZ2, dZ1,
                     loss_sum, correct);
  return hipGetLastError();
}

hipError_t pde_lenet_head_bwd(const float* H1, int B, const float* W2, const float* logp, const float* g, float* dZ2,
                              float* dZ1, hipStream_t st) {
  hipLaunchKernelGGL(k_head_bwd, dim3((B + 3) / 4), dim3(256), 0, st, H1, B, W2, logp, g, dZ2, dZ1);
  return hipGetLastError();
}

hipError_t pde_lenet_fc_bwd(const float* P2, const float* H1, const float* dZ1, const float* dZ2, const float* W1,
                            int B, float* dP2m, float* gW1, float* gb1, float* gW2, float* gb2, hipStream_t st) {
  const int nblk = ((B + 15) / 16) * 50 + 32 * 13 + 8;
  hipLaunchKernelGGL(k_fc_bwd, dim3(nblk), dim3(256), 0, st, P2, H1, dZ1, dZ2, W1, B, dP2m, gW1, gb1, gW2, gb2);
  return hipGetLastError();
}

hipError_t pde_lenet_conv_bwd(const float* X, const int* rows, const float* P1, const uint8_t* A1,
                              const float* dP2m, const uint8_t* A2, const float* W2c, int B, float* gW1c,
                              float* gb1c, float* gW2c, float* gb2c, hipStream_t st) {
  const int nblk = ((B + kWImgs - 1) / kWImgs) * 8 + 4 * B;
  hipLaunchKernelGGL(k_conv_bwd, dim3(nblk), dim3(256), 0, st, X, rows, P1, A1, dP2m, A2, W2c, B, gW1c, gb1c,
                     gW2c, gb2c);
  return hipGetLastError();
}

}  // extern "C"
