// ResNet kernels for gfx950: training-mode BatchNorm over NHWC bf16 activations fused with the
// residual add and ReLU (forward: stats -> finalize -> apply; backward: reduce -> finalize -> apply),
// and the SGD(momentum) step on bf16 weights with fp32 master weights.
//
// NHWC = rows of C channels.  A 256-thread block owns a contiguous row range; thread t handles the
// 8-channel chunk t % (C/8) of rows t / (C/8) + k*RP (RP = 256 / (C/8)), so per-channel partial sums
// stay in registers and one LDS pass folds the RP row-lanes.  Partials [nblk][2C] are reduced by a
// per-channel finalize kernel that also produces the fused per-channel coefficients of the apply
// pass (y = x*scale + shift (+res), relu; dx = A*dy' + B*x + Cc, dy' = dy*(y>0)).
#include "pde_hip.h"
#include "pde_bf16.h"
#include "pde_kernels.h"

namespace {

__device__ __forceinline__ void bn_geom(int C, int& CP, int& RP) {
  CP = C >> 3;
  RP = 256 / CP;
}

// ------------------------------------------------------------------------------- forward stats
__global__ __launch_bounds__(256) void k_bn_stats(const uint4* __restrict__ X, int M, int C, int rows_per_block,
                                                  float* __restrict__ part) {
  extern __shared__ float sh[];  // [RP][2][C]
  int CP, RP;
  bn_geom(C, CP, RP);
  const int tid = threadIdx.x, c8 = tid % CP, rl = tid / CP;
  float s[8], q[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rl < RP) {
    int r = r0 + rl;
    for (; r + RP < r1; r += 2 * RP) {  // two rows in flight
      float v[8], w[8];
      unpack8(X[(size_t)r * CP + c8], v);
      unpack8(X[(size_t)(r + RP) * CP + c8], w);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[e] += v[e] + w[e];
        q[e] += v[e] * v[e] + w[e] * w[e];
      }
    }
    for (; r < r1; r += RP) {
      float v[8];
      unpack8(X[(size_t)r * CP + c8], v);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[e] += v[e];
        q[e] += v[e] * v[e];
      }
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sh[(rl * 2 + 0) * C + c8 * 8 + e] = s[e];
      sh[(rl * 2 + 1) * C + c8 * 8 + e] = q[e];
    }
  }
  __syncthreads();
  for (int k = tid; k < 2 * C; k += 256) {
    const int which = k / C, c = k % C;
    float t = 0.f;
    for (int j = 0; j < RP; ++j) t += sh[(j * 2 + which) * C + c];
    part[(size_t)blockIdx.x * 2 * C + k] = t;
  }
}

// Sum the [nblk][2C] partials of the 64 channels [64*blockIdx.x, +64): 1024 threads = 64 channel
// lanes x 16 waves striding over the partial rows, LDS fold.  Each lane keeps 8 rows (16 loads) in
// flight (these folds are latency-bound: with 2 in flight, 512 rows cost 16 dependent round trips, ~7 us).
__device__ __forceinline__ void fold_partials(const float* __restrict__ part, int nblk, int C, int c, float& s,
                                              float& q) {
  __shared__ float sh[16][2][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int cc = min(c, C - 1);
  // 8 rows (16 loads) in flight per lane: 512 partial rows are 4 dependent round trips, not 8
  float sa[8], qa[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) sa[u] = qa[u] = 0.f;
  int b = w;
  for (; b + 112 < nblk; b += 128) {
    float sv[8], qv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sv[u] = part[(size_t)(b + 16 * u) * 2 * C + cc];
      qv[u] = part[(size_t)(b + 16 * u) * 2 * C + C + cc];
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sa[u] += sv[u];
      qa[u] += qv[u];
    }
  }
  {
    // remainder (< 128 rows): up to 8 rows per wave, all loads issued before any is summed
    float sv[8], qv[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int r = b + 16 * u;
      sv[u] = r < nblk ? part[(size_t)r * 2 * C + cc] : 0.f;
      qv[u] = r < nblk ? part[(size_t)r * 2 * C + C + cc] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      sa[u] += sv[u];
      qa[u] += qv[u];
    }
  }
  sh[w][0][lane] = ((sa[0] + sa[1]) + (sa[2] + sa[3])) + ((sa[4] + sa[5]) + (sa[6] + sa[7]));
  sh[w][1][lane] = ((qa[0] + qa[1]) + (qa[2] + qa[3])) + ((qa[4] + qa[5]) + (qa[6] + qa[7]));
  __syncthreads();
  s = 0.f;
  q = 0.f;
  if (w == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      s += sh[k][0][lane];
      q += sh[k][1][lane];
    }
  }
}

// out[y][c] = sum of partial rows [y*rows_per, (y+1)*rows_per) of part[nblk][W]: folds the many
// per-tile partials of a conv epilogue (thousands of rows) before the per-channel finalize
// (16 rows in flight per thread).
__global__ __launch_bounds__(256) void k_fold_rows(const float* __restrict__ part, int nblk, int W, int rows_per,
                                                   float* __restrict__ out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= W) return;
  const int r0 = blockIdx.y * rows_per, r1 = min(nblk, r0 + rows_per);
  float a[16];
#pragma unroll
  for (int u = 0; u < 16; ++u) a[u] = 0.f;
  int r = r0;
  for (; r + 15 < r1; r += 16) {       // 16 rows in flight: 56 rows (B = 256 layer1) in 4 round trips
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = part[(size_t)(r + u) * W + c];
#pragma unroll
    for (int u = 0; u < 16; ++u) a[u] += v[u];
  }
  {
    float v[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) v[u] = r + u < r1 ? part[(size_t)(r + u) * W + c] : 0.f;
#pragma unroll
    for (int u = 0; u < 16; ++u) a[u] += v[u];
  }
#pragma unroll
  for (int u = 0; u < 8; ++u) a[u] += a[u + 8];
  out[(size_t)blockIdx.y * W + c] = ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// per channel: mean / biased var -> rstd, running-stat update (unbiased var), scale / shift
__global__ __launch_bounds__(1024) void k_bn_finalize(const float* __restrict__ part, int nblk, int C, int M,
                                                      const bf16_t* __restrict__ gamma,
                                                      const bf16_t* __restrict__ beta, float eps, float momentum,
                                                      float* __restrict__ run_mean, float* __restrict__ run_var,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                      float* __restrict__ scale, float* __restrict__ shift) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float s, q;
  fold_partials(part, nblk, C, c, s, q);
  if (threadIdx.x >= 64 || c >= C) return;
  const float mean = s / M;
  const float var = fmaxf(q / M - mean * mean, 0.f);
  const float rstd = rsqrtf(var + eps);
  if (run_mean) {
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * var * ((float)M / (float)max(M - 1, 1));
  }
  mean_out[c] = mean;
  rstd_out[c] = rstd;
  const float g = bf2f(gamma[c]), bt = bf2f(beta[c]);
  scale[c] = g * rstd;
  shift[c] = bt - mean * g * rstd;
}

// y = x*scale + shift (+ res), optional relu.  The grid stride is a multiple of C/8, so each
// thread's channel chunk is fixed: its 8 scale / shift values are loaded once.
// rscale / rshift (optional): the residual is itself a BatchNorm input (a ResNet downsample branch,
// bn_d(conv_d(x))), applied here as res*rscale + rshift -- the branch's normalised tensor is never
// written and read back (one rounding instead of two)
__global__ __launch_bounds__(256) void k_bn_apply(const uint4* __restrict__ X, const uint4* __restrict__ R,
                                                  const float* __restrict__ scale, const float* __restrict__ shift,
                                                  const float* __restrict__ rscale, const float* __restrict__ rshift,
                                                  uint4* __restrict__ Y, int64_t n8, int CP, int relu) {
  const int64_t i0 = blockIdx.x * 256ll + threadIdx.x;
  const int c0 = (int)(i0 & (CP - 1)) * 8;
  float sc[8], sf[8], rc[8], rf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[c0 + e];
    sf[e] = shift[c0 + e];
    rc[e] = 1.f;
    rf[e] = 0.f;
  }
  // one uniform branch around the vector loads (a per-element pointer-or-constant select became 16
  // scalar loads behind branches: a prologue of dependent round trips that doubled the pass time)
  if (rscale) {
    const float4* a = reinterpret_cast<const float4*>(rscale + c0);
    const float4* b = reinterpret_cast<const float4*>(rshift + c0);
    const float4 a0 = a[0], a1 = a[1], b0 = b[0], b1 = b[1];
    rc[0] = a0.x; rc[1] = a0.y; rc[2] = a0.z; rc[3] = a0.w; rc[4] = a1.x; rc[5] = a1.y; rc[6] = a1.z; rc[7] = a1.w;
    rf[0] = b0.x; rf[1] = b0.y; rf[2] = b0.z; rf[3] = b0.w; rf[4] = b1.x; rf[5] = b1.y; rf[6] = b1.z; rf[7] = b1.w;
  }
  for (int64_t i = i0; i < n8; i += (int64_t)gridDim.x * 256) {
    float v[8], r[8];
    unpack8(X[i], v);
    if (R) unpack8(R[i], r);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float o = v[e] * sc[e] + sf[e] + (R ? r[e] * rc[e] + rf[e] : 0.f);
      v[e] = relu ? fmaxf(o, 0.f) : o;
    }
    Y[i] = pack8(v);
  }
}

// ------------------------------------------------------------------------------- backward
// part[blk] = (sum dy', sum dy' * xhat) per channel, dy' = dy * (y > 0) when relu
// relu: 0 none, 1 mask from the saved output Y (y > 0), 2 mask recomputed from the input X with the
// forward's per-channel scale / shift (x*scale + shift > 0; no residual): one tensor less to read
// (a template parameter: a runtime mode made the per-thread prologue heavy enough to slow the small
// layer4 passes 4x)
__device__ __forceinline__ void load8f(const float* __restrict__ p, float* v) {
  const float4 a = *reinterpret_cast<const float4*>(p), b = *reinterpret_cast<const float4*>(p + 4);
  v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}

template <int RELU>
__global__ __launch_bounds__(256) void k_bn_bwd_reduce(const uint4* __restrict__ dY, const uint4* __restrict__ Y,
                                                       const uint4* __restrict__ X, const float* __restrict__ mean,
                                                       const float* __restrict__ rstd, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, int M, int C,
                                                       int rows_per_block, float* __restrict__ part,
                                                       uint4* __restrict__ dR) {
  extern __shared__ float sh[];
  int CP, RP;
  bn_geom(C, CP, RP);
  const int tid = threadIdx.x, c8 = tid % CP, rl = tid / CP;
  float s[8], q[8], mu[8], rs[8], sc[8], sf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  load8f(mean + c8 * 8, mu);
  load8f(rstd + c8 * 8, rs);
  if constexpr (RELU == 2) {
    load8f(scale + c8 * 8, sc);
    load8f(shift + c8 * 8, sf);
  }
  const int r0 = blockIdx.x * rows_per_block, r1 = min(M, r0 + rows_per_block);
  if (rl < RP) {
    for (int r = r0 + rl; r < r1; r += RP) {
      const size_t i = (size_t)r * CP + c8;
      float g[8], x[8], y[8];
      unpack8(dY[i], g);
      unpack8(X[i], x);
      if constexpr (RELU == 1) unpack8(Y[i], y);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        float d = g[e];
        if constexpr (RELU == 1) d = y[e] > 0.f ? d : 0.f;
        if constexpr (RELU == 2) d = x[e] * sc[e] + sf[e] > 0.f ? d : 0.f;
        s[e] += d;
        q[e] += d * (x[e] - mu[e]) * rs[e];
        g[e] = d;
      }
      if (RELU == 1 && dR) dR[i] = pack8(g);   // the residual gradient IS the masked gradient
    }
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sh[(rl * 2 + 0) * C + c8 * 8 + e] = s[e];
      sh[(rl * 2 + 1) * C + c8 * 8 + e] = q[e];
    }
  }
  __syncthreads();
  for (int k = tid; k < 2 * C; k += 256) {
    const int which = k / C, c = k % C;
    float t = 0.f;
    for (int j = 0; j < RP; ++j) t += sh[(j * 2 + which) * C + c];
    part[(size_t)blockIdx.x * 2 * C + k] = t;
  }
}

// dgamma = sum dy'*xhat, dbeta = sum dy'; dx = A*dy' + B*x + Cc with A = g*rstd,
// B = -A*rstd*mean(dy'xhat), Cc = -A*mean(dy') - B*mean
__global__ __launch_bounds__(1024) void k_bn_bwd_finalize(const float* __restrict__ part, int nblk, int C, int M,
                                                          const bf16_t* __restrict__ gamma,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ rstd,
                                                          bf16_t* __restrict__ dgamma, bf16_t* __restrict__ dbeta,
                                                          float* __restrict__ coef) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  float s, q;
  fold_partials(part, nblk, C, c, s, q);
  if (threadIdx.x >= 64 || c >= C) return;
  dgamma[c] = f2bf(q);
  dbeta[c] = f2bf(s);
  const float A = bf2f(gamma[c]) * rstd[c];
  const float Bc = -A * rstd[c] * (q / M);
  coef[c] = A;
  coef[C + c] = Bc;
  coef[2 * C + c] = -A * (s / M) - Bc * mean[c];
}

template <int RELU>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const uint4* __restrict__ dY, const uint4* __restrict__ Y,
                                                      const uint4* __restrict__ X, const float* __restrict__ coef,
                                                      const float* __restrict__ scale, const float* __restrict__ shift,
                                                      uint4* __restrict__ dX, uint4* __restrict__ dR, int64_t n8,
                                                      int C) {
  const int CP = C >> 3;
  const int64_t i0 = blockIdx.x * 256ll + threadIdx.x;
  const int c0 = (int)(i0 & (CP - 1)) * 8;
  float ca[8], cb[8], cc[8], sc[8], sf[8];
  load8f(coef + c0, ca);
  load8f(coef + C + c0, cb);
  load8f(coef + 2 * C + c0, cc);
  if constexpr (RELU == 2) {
    load8f(scale + c0, sc);
    load8f(shift + c0, sf);
  }
  for (int64_t i = i0; i < n8; i += (int64_t)gridDim.x * 256) {
    float g[8], x[8], y[8], o[8];
    unpack8(dY[i], g);
    unpack8(X[i], x);
    if constexpr (RELU == 1) unpack8(Y[i], y);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float d = g[e];
      if constexpr (RELU == 1) d = y[e] > 0.f ? d : 0.f;
      if constexpr (RELU == 2) d = x[e] * sc[e] + sf[e] > 0.f ? d : 0.f;
      g[e] = d;
      o[e] = ca[e] * d + cb[e] * x[e] + cc[e];
    }
    dX[i] = pack8(o);
    if (dR) dR[i] = pack8(g);
  }
}

// ------------------------------------------------------------------------------- max-pool 3x3 / 2, pad 1
// NHWC bf16.  Forward keeps the window argmax (0..8, first maximum in scan order like ATen) as one
// byte per element; backward GATHERS: each input element sums the <= 2x2 windows that cover it and
// chose it -- no atomics.
__global__ __launch_bounds__(256) void k_maxpool3s2_fwd(const uint4* __restrict__ X, uint4* __restrict__ Y,
                                                        uint2* __restrict__ A, int N, int H, int W, int OH, int OW,
                                                        int CP) {
  const int64_t total = (int64_t)N * OH * OW * CP;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(t % CP);
    int64_t p = t / CP;
    const int ow = (int)(p % OW);
    p /= OW;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    float best[8];
    uint32_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      arg[e] = 0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        const bool ok = ih >= 0 && ih < H && iw >= 0 && iw < W;
        const int ihc = min(max(ih, 0), H - 1), iwc = min(max(iw, 0), W - 1);
        float v[8];
        unpack8(X[(((int64_t)n * H + ihc) * W + iwc) * CP + c8], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const bool better = ok && v[e] > best[e];
          best[e] = better ? v[e] : best[e];
          arg[e] = better ? (uint32_t)(kh * 3 + kw) : arg[e];
        }
      }
    }
    Y[t] = pack8(best);
    A[t] = make_uint2(arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24),
                      arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24));
  }
}

__global__ __launch_bounds__(256) void k_maxpool3s2_bwd(const uint4* __restrict__ dY, const uint2* __restrict__ A,
                                                        uint4* __restrict__ dX, int N, int H, int W, int OH, int OW,
                                                        int CP) {
  const int64_t total = (int64_t)N * H * W * CP;
  for (int64_t t = blockIdx.x * 256ll + threadIdx.x; t < total; t += (int64_t)gridDim.x * 256) {
    const int c8 = (int)(t % CP);
    int64_t p = t / CP;
    const int iw = (int)(p % W);
    p /= W;
    const int ih = (int)(p % H);
    const int n = (int)(p / H);
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    const int oh0 = ih / 2, ow0 = iw / 2;  // candidates: oh in {oh0, oh0 + 1 if ih odd}, same for ow
#pragma unroll
    for (int a = 0; a < 2; ++a) {
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int oh = oh0 + a, ow = ow0 + b;
        const bool ok = (a == 0 || (ih & 1)) && (b == 0 || (iw & 1)) && oh < OH && ow < OW;
        const int ohc = min(oh, OH - 1), owc = min(ow, OW - 1);
        const int64_t o = (((int64_t)n * OH + ohc) * OW + owc) * CP + c8;
        float g[8];
        unpack8(dY[o], g);
        const uint2 ar = A[o];
        const uint32_t want = (uint32_t)((ih - (2 * ohc - 1)) * 3 + (iw - (2 * owc - 1)));
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const uint32_t ae = ((e < 4 ? ar.x : ar.y) >> (8 * (e & 3))) & 0xffu;
          acc[e] += (ok && ae == want) ? g[e] : 0.f;
        }
      }
    }
    dX[t] = pack8(acc);
  }
}

// ------------------------------------------------------------------------------- stem BN + ReLU + max-pool
// The stem's BatchNorm apply, ReLU and 3x3/s2/p1 max-pool as ONE pass over the conv output y: the
// post-BN map a = relu(y*scale + shift) (411 MB at B=256) is never materialised.  Forward writes only
// the pooled map and its window argmax; backward recomputes a's sign from y and runs two passes over y:
//   REDUCE: d = pooling gather of dP (each input element sums the <= 2x2 windows that chose it) masked
//           by a > 0, then the BN partials (sum d, sum d*xhat) -> part[blk][2][C]
//   APPLY:  the same d, dy = A*d + B*y + Cc (coefficients of k_bn_bwd_finalize)
// replacing bn_apply + maxpool fwd and maxpool bwd + bn_bwd_reduce + bn_bwd_apply (5 full passes, 2 of
// them writing 411 MB).  One block per pooled row (fwd) / per rows_per_block input rows (bwd) of one
// image, so the row index needs no division; blockDim is a multiple of CP (a thread's channel chunk is
// fixed) and a thread walks the row's (column, chunk) pairs.
__global__ __launch_bounds__(512) void k_bnpool_fwd(const uint4* __restrict__ Y, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, uint4* __restrict__ P,
                                                    uint2* __restrict__ Arg, uint4* __restrict__ Ysel, int H, int W,
                                                    int OH, int OW, int CP, int lgcp) {
  const int oh = blockIdx.x, n = blockIdx.y, c8 = threadIdx.x & (CP - 1);
  float sc[8], sf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[c8 * 8 + e];
    sf[e] = shift[c8 * 8 + e];
  }
  const uint4* yimg = Y + (size_t)n * H * W * CP;
  for (int idx = threadIdx.x; idx < OW * CP; idx += blockDim.x) {
    const int ow = idx >> lgcp;
    float best[8], ysel[8];
    uint32_t arg[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      best[e] = -INFINITY;
      ysel[e] = 0.f;
      arg[e] = 0;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - 1 + kh;
      if (ih < 0 || ih >= H) continue;  // uniform over the block
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - 1 + kw;
        const bool ok = iw >= 0 && iw < W;
        float v[8];
        unpack8(yimg[(ih * W + min(max(iw, 0), W - 1)) * CP + c8], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          // the value the unfused path pooled: relu(bn(y)) rounded to bf16 (same ties, same argmax)
          const float a = bf2f(f2bf(fmaxf(v[e] * sc[e] + sf[e], 0.f)));
          const bool better = ok && a > best[e];
          best[e] = better ? a : best[e];
          ysel[e] = better ? v[e] : ysel[e];
          arg[e] = better ? (uint32_t)(kh * 3 + kw) : arg[e];
        }
      }
    }
    const size_t o = ((size_t)(n * OH + oh) * OW + ow) * CP + c8;
    P[o] = pack8(best);
    Ysel[o] = pack8(ysel);
    Arg[o] = make_uint2(arg[0] | (arg[1] << 8) | (arg[2] << 16) | (arg[3] << 24),
                        arg[4] | (arg[5] << 8) | (arg[6] << 16) | (arg[7] << 24));
  }
}

// The same fused apply + pool with one thread per 2 x JW block of pooled cells (oh0 + i, ow0 + j) and
// chunk: the 5 x (2 JW + 1) input patch rows 2 oh0 - 1 .. 2 oh0 + 3, columns 2 ow0 - 1 .. 2 ow0 + 2 JW - 1
// covers all its windows, so (JW = 2) a thread issues 25 16-byte loads and 25 relu(bn(.)) evaluations
// for 4 outputs instead of 36 + 36 (JW = 1: 15 for 2).  The patch streams row by row (5 loads in flight); each element updates the windows
// that contain it in the same (kh, kw) order as k_bnpool_fwd, so ties resolve identically.
template <int JW>
__global__ __launch_bounds__(256) void k_bnpool_fwd2(const uint4* __restrict__ Y, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, uint4* __restrict__ P,
                                                     uint2* __restrict__ Arg, uint4* __restrict__ Ysel, int H, int W,
                                                     int OH, int OW, int CP, int lgcp) {
  const int oh0 = 2 * blockIdx.x, n = blockIdx.y, c8 = threadIdx.x & (CP - 1);
  constexpr int NC = 2 * JW + 1, NQ = 2 * JW;   // patch columns, outputs per thread
  const int owp = (OW + JW - 1) / JW;
  float sc[8], sf[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    sc[e] = scale[c8 * 8 + e];
    sf[e] = shift[c8 * 8 + e];
  }
  const uint4* yimg = Y + (size_t)n * H * W * CP;
  for (int idx = threadIdx.x; idx < owp * CP; idx += blockDim.x) {
    const int ow0 = JW * (idx >> lgcp);
    float best[NQ][8], ysel[NQ][8];
    uint32_t arg[NQ][8];
#pragma unroll
    for (int q = 0; q < NQ; ++q)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        best[q][e] = -INFINITY;
        ysel[q][e] = 0.f;
        arg[q][e] = 0;
      }
#pragma unroll
    for (int r = 0; r < 5; ++r) {
      const int ih = 2 * oh0 - 1 + r;
      if (ih < 0 || ih >= H) continue;  // uniform over the block
      uint4 raw[NC];
#pragma unroll
      for (int c = 0; c < NC; ++c) raw[c] = yimg[(ih * W + min(max(2 * ow0 - 1 + c, 0), W - 1)) * CP + c8];
#pragma unroll
      for (int c = 0; c < NC; ++c) {
        const int iw = 2 * ow0 - 1 + c;
        const bool ok = iw >= 0 && iw < W;
        float v[8];
        unpack8(raw[c], v);
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float a = bf2f(f2bf(fmaxf(v[e] * sc[e] + sf[e], 0.f)));
#pragma unroll
          for (int i = 0; i < 2; ++i) {
            if (r < 2 * i || r > 2 * i + 2) continue;  // compile-time after unrolling
#pragma unroll
            for (int j = 0; j < JW; ++j) {
              if (c < 2 * j || c > 2 * j + 2) continue;
              const int q = JW * i + j;
              const bool better = ok && a > best[q][e];
              best[q][e] = better ? a : best[q][e];
              ysel[q][e] = better ? v[e] : ysel[q][e];
              arg[q][e] = better ? (uint32_t)((r - 2 * i) * 3 + c - 2 * j) : arg[q][e];
            }
          }
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const int oh = oh0 + q / JW, ow = ow0 + q % JW;
      if (oh >= OH || ow >= OW) continue;
      const size_t o = ((size_t)(n * OH + oh) * OW + ow) * CP + c8;
      P[o] = pack8(best[q]);
      Ysel[o] = pack8(ysel[q]);
      Arg[o] = make_uint2(arg[q][0] | (arg[q][1] << 8) | (arg[q][2] << 16) | (arg[q][3] << 24),
                          arg[q][4] | (arg[q][5] << 8) | (arg[q][6] << 16) | (arg[q][7] << 24));
    }
  }
}

// Backward.  The BN partials need only the windows: d is non-zero only where a window took its
// maximum, so sum d = sum over windows of dP (masked by a > 0) and sum d*y = sum over windows of
// dP * y[argmax].  The forward stores y[argmax] (Ysel, one pooled map), and the reduce pass is
// k_bn_bwd_reduce<2> over (dP, Ysel) -- its ReLU mask ysel*scale + shift > 0 is the apply pass's mask
// at the argmax element -- reading 2 pooled maps instead of dP, the argmax and all of y (565 -> 206 MB
// at B = 256; the former gather pass took 200 us).
// The apply pass, one thread per POOLED cell (oh, ow, chunk) handling the 2x2 input block
// (2oh + i, 2ow + j): an even input row / column is covered by window oh / ow only, an odd one by oh
// and oh + 1, so the four windows {oh, oh+1} x {ow, ow+1} serve all four input elements.  A block
// covers RB pooled rows (2 RB input rows) and cols_per pooled columns (blockIdx.z-th column block) of
// one image with one thread per (column, chunk):
//  * the RB + 1 pooled gradient / argmax rows it needs (one halo row) over its columns + one halo
//    column are staged in LDS once with 16-byte loads, and the four windows of a cell are LDS reads;
//  * column blocks of <= 256 threads: at 158 VGPRs a CU holds 12 waves, i.e. one whole-row block of
//    7 waves but three 4-wave half-row blocks;
//  * a thread's input chunks (y) of the next two row pairs are in flight while the current pair computes;
//  * dy = A*d + B*y + Cc with d the pooling gather of dP masked by a > 0.
template <int RB>
__global__ __launch_bounds__(256, 3) void k_bnpool_bwd(const uint4* __restrict__ dP, const uint2* __restrict__ Arg,
                                                       const uint4* __restrict__ Y, const float* __restrict__ scale,
                                                       const float* __restrict__ shift, const float* __restrict__ coef,
                                                       uint4* __restrict__ dY, int H, int W, int OH, int OW, int CP,
                                                       int lgcp, int cols_per) {
  extern __shared__ __attribute__((aligned(16))) char bsm[];
  const int ncell = OW * CP;                            // cells of a pooled row
  const int c_lo = blockIdx.z * cols_per, c_hi = min(OW, c_lo + cols_per);
  if (c_lo >= OW) return;                               // whole block
  const int sw = min(c_hi + 1, OW) - c_lo;              // staged columns (incl. the halo column)
  const int scell = sw * CP;
  uint4* gs = reinterpret_cast<uint4*>(bsm);           // [RB + 1][scell] pooled gradient chunks
  uint2* as = reinterpret_cast<uint2*>(bsm + (size_t)(RB + 1) * (cols_per + 1) * CP * 16);   // argmax codes
  const int n = blockIdx.y, t = threadIdx.x, c8 = t & (CP - 1), C = CP * 8;
  const int r0 = blockIdx.x * RB;
  const int nrow = min(RB + 1, OH - r0);               // staged pooled rows (incl. the halo row)
  const uint4* dimg = dP + ((size_t)n * OH + r0) * ncell + c_lo * CP;
  const uint2* aimg = Arg + ((size_t)n * OH + r0) * ncell + c_lo * CP;
  for (int e = t; e < nrow * scell; e += blockDim.x) {
    const int row = e / scell, x = e - row * scell;
    gs[e] = dimg[row * ncell + x];
    as[e] = aimg[row * ncell + x];
  }
  float sc[8], sf[8], k0[8], k1[8], k2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    const int c = c8 * 8 + e;
    sc[e] = scale[c];
    sf[e] = shift[c];
    k0[e] = coef[c];
    k1[e] = coef[C + c];
    k2[e] = coef[2 * C + c];
  }
  const bool live = t < (c_hi - c_lo) * CP;
  const int cell = live ? t : 0, ow = c_lo + (cell >> lgcp);
  // the thread's input chunks of a row pair (zeros past the image); the next two pairs' are loaded
  // while the current one is processed
  auto load_y = [&](int r, uint4 (&v)[2][2]) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int ih = 2 * (r0 + r) + i, iw = 2 * ow + j;
        v[i][j] = make_uint4(0u, 0u, 0u, 0u);
        if (live && r0 + r < OH && ih < H && iw < W) v[i][j] = Y[((size_t)(n * H + ih) * W + iw) * CP + c8];
      }
  };
  constexpr int PRE = 2;
  uint4 yv[RB][2][2], ycur[2][2];
#pragma unroll
  for (int r = 0; r <= PRE && r < RB; ++r) load_y(r, yv[r]);
  __syncthreads();
  const bool bok = ow + 1 < OW;
#pragma unroll
  for (int r = 0; r < RB; ++r) {
    const int oh = r0 + r;
    if (r > 0 && r + PRE < RB) load_y(r + PRE, yv[r + PRE]);
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) ycur[i][j] = yv[r][i][j];
    if (!live || oh >= OH) continue;
    const bool aok = oh + 1 < OH;
    uint4 g[2][2];                                     // window gradients, packed bf16
    uint2 ar[2][2];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int rr = min(r + a, nrow - 1), oc = min(ow + b, OW - 1);
        const int o = rr * scell + (oc - c_lo) * CP + c8;
        g[a][b] = gs[o];
        ar[a][b] = as[o];
      }
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int ih = 2 * oh + i;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int iw = 2 * ow + j;
        if (ih >= H || iw >= W) continue;
        float y[8];
        unpack8(ycur[i][j], y);
        float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int a = 0; a < 2; ++a) {
          if (a > i) continue;                       // window row oh+1 covers odd rows only
#pragma unroll
          for (int b = 0; b < 2; ++b) {
            if (b > j) continue;
            const bool ok = (a == 0 || aok) && (b == 0 || bok);
            const uint32_t want = (uint32_t)((i - 2 * a + 1) * 3 + (j - 2 * b + 1));
            float gv[8];
            unpack8(g[a][b], gv);
#pragma unroll
            for (int e = 0; e < 8; ++e) {
              const uint32_t ae = ((e < 4 ? ar[a][b].x : ar[a][b].y) >> (8 * (e & 3))) & 0xffu;
              acc[e] += (ok && ae == want) ? gv[e] : 0.f;
            }
          }
        }
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float d = (y[e] * sc[e] + sf[e] > 0.f) ? acc[e] : 0.f;
          acc[e] = k0[e] * d + k1[e] * y[e] + k2[e];
        }
        dY[((size_t)(n * H + ih) * W + iw) * CP + c8] = pack8(acc);
      }
    }
  }
}

// ------------------------------------------------------------------------------- SGD (master)
// torch.optim.SGD semantics (coupled weight decay, dampening 0): g' = g*s + wd*p; buf = mom*buf + g'
// (buf starts at 0, which equals torch's buf = g' on the first step); p -= lr * (nesterov ? g' + mom*buf : buf)
__global__ __launch_bounds__(256) void k_sgd_master(float* __restrict__ master, uint2* __restrict__ p16,
                                                    const uint2* __restrict__ g16, float4* __restrict__ buf, int64_t n4,
                                                    float lr, float momentum, float wd, int nesterov, float grad_scale,
                                                    const uint8_t* __restrict__ decay_blk) {
  float4* mp = reinterpret_cast<float4*>(master);
  for (int64_t i = blockIdx.x * 256ll + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256) {
    float4 p = mp[i], b = buf[i];
    float g[4];
    unpack4(g16[i], g);
    const float w = (decay_blk == nullptr || decay_blk[i >> 4]) ? wd : 0.f;
    float* pp = &p.x;
    float* bb = &b.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gg = g[e] * grad_scale + w * pp[e];
      bb[e] = momentum * bb[e] + gg;
      pp[e] -= lr * (nesterov ? gg + momentum * bb[e] : bb[e]);
    }
    mp[i] = p;
    buf[i] = b;
    p16[i] = pack4(pp);
  }
}

inline int grid_cap(int64_t n, int cap) {
  int64_t g = (n + 255) / 256;
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

// ---- global average pool over NHWC (the ResNet head before the FC GEMM) ----
// fwd: out[n][c] = mean_hw x[n][hw][c]; one thread per (n, 8-channel chunk), fp32 sum
__global__ __launch_bounds__(256) void k_avgpool_fwd(const uint4* __restrict__ x, uint4* __restrict__ out, int N,
                                                     int HW, int C8, float inv) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= N * C8) return;
  const int n = i / C8, c = i - n * C8;
  float s[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int p = 0; p < HW; ++p) {
    float v[8];
    unpack8(x[((size_t)n * HW + p) * C8 + c], v);
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] += v[e];
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) s[e] *= inv;
  out[i] = pack8(s);
}
// bwd: dx[n][hw][c] = dout[n][c] / HW
__global__ __launch_bounds__(256) void k_avgpool_bwd(const uint4* __restrict__ dout, uint4* __restrict__ dx, int N,
                                                     int HW, int C8, float inv) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= (int64_t)N * HW * C8) return;
  const int c = (int)(i % C8);
  const int n = (int)(i / ((int64_t)HW * C8));
  float v[8];
  unpack8(dout[(size_t)n * C8 + c], v);
#pragma unroll
  for (int e = 0; e < 8; ++e) v[e] *= inv;
  dx[i] = pack8(v);
}

}  // namespace

extern "C" {

int pde_bn_blocks(int M, int C) {
  // ~2 blocks per CU, each at least a few row-lane strides long
  const int rp = 256 / (C / 8);
  int nblk = 512;
  const int min_rows = rp * 8;
  if ((M + nblk - 1) / nblk < min_rows) nblk = (M + min_rows - 1) / min_rows;
  return nblk < 1 ? 1 : nblk;
}

constexpr int kFoldThreshold = 256, kFoldRows = 64;
int pde_bn_part_rows(int pre_nblk) { return pre_nblk > kFoldThreshold ? pre_nblk + kFoldRows : pre_nblk; }

// res_scale / res_shift (optional, with res): the residual is normalised on the fly (k_bn_apply)
hipError_t pde_bn_fwd(const void* x, const void* res, void* y, int M, int C, const void* gamma, const void* beta,
                      float eps, float momentum, float* run_mean, float* run_var, float* part, float* mean,
                      float* rstd, float* scale, float* shift, int relu, int training, int pre_nblk,
                      const float* res_scale, const float* res_shift, hipStream_t st) {
  if ((res_scale || res_shift) && (!res || !res_scale || !res_shift)) return hipErrorInvalidValue;
  if (C % 8 != 0 || 256 % (C / 8) != 0) return hipErrorInvalidValue;
  const int CP = C / 8, RP = 256 / CP;
  if (training) {
    // pre_nblk > 0: `part` already holds [pre_nblk][2][C] partial sums (the producing convolution's
    // epilogue, conv.hip), so the statistics pass over x is skipped
    int nblk = pre_nblk > 0 ? pre_nblk : pde_bn_blocks(M, C);
    const int rpb = (M + nblk - 1) / nblk;
    if (pre_nblk <= 0)
      hipLaunchKernelGGL(k_bn_stats, dim3(nblk), dim3(256), (size_t)RP * 2 * C * sizeof(float), st,
                         (const uint4*)x, M, C, rpb, part);
    if (pre_nblk > kFoldThreshold) {
      // too many partial rows for the finalize's per-channel fold: pre-fold into kFoldRows rows
      // stored after them (the caller sizes part as (pre_nblk + kFoldRows) x 2C)
      float* folded = part + (size_t)pre_nblk * 2 * C;
      const int rows_per = (pre_nblk + kFoldRows - 1) / kFoldRows;
      hipLaunchKernelGGL(k_fold_rows, dim3((2 * C + 255) / 256, kFoldRows), dim3(256), 0, st, part, pre_nblk,
                         2 * C, rows_per, folded);
      part = folded;
      nblk = kFoldRows;
    }
    hipLaunchKernelGGL(k_bn_finalize, dim3((C + 63) / 64), dim3(1024), 0, st, part, nblk, C, M,
                       (const bf16_t*)gamma, (const bf16_t*)beta, eps, momentum, run_mean, run_var, mean, rstd, scale,
                       shift);
  }
  const int64_t n8 = (int64_t)M * CP;
  if (y)   // y == nullptr: statistics / finalize only (the apply is fused into a consumer, e.g. k_bnpool_fwd)
    hipLaunchKernelGGL(k_bn_apply, dim3(grid_cap(n8, 4096)), dim3(256), 0, st, (const uint4*)x, (const uint4*)res,
                       scale, shift, res_scale, res_shift, (uint4*)y, n8, CP, relu);
  return hipGetLastError();
}

// fused stem BN + ReLU + max-pool (k_bnpool_*): launch geometry shared by the host functions below
static int bnpool_threads(int cols_cp) {
  const int iters = (cols_cp + 511) / 512;
  return ((cols_cp + iters - 1) / iters + 63) / 64 * 64;
}
constexpr int kBnpoolRB = 4;            // pooled rows per backward block
static int ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return l;
}

// blocks of the backward passes: kBnpoolRB pooled rows (2 kBnpoolRB input rows) of one image
int pde_bnpool_part_floats(int N, int H, int W, int C) {
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  return pde_bn_part_rows(pde_bn_blocks(N * OH * OW, C)) * 2 * C;
}

hipError_t pde_bnpool_fwd(const void* y, const float* scale, const float* shift, void* p, void* arg, void* ysel,
                          int N, int C, int H, int W, int OH, int OW, hipStream_t st) {
  const int CP = C / 8;
  if (C % 8 || (CP & (CP - 1)) || CP > 64) return hipErrorInvalidValue;
  // pooled cells per thread: 1, 2 (vertical pair, the default) or 4 (2x2 block); read per call (once
  // per step) so that a test can compare the variants in one process.  ResNet-18 stem at B = 256
  // (profiles/r5_models/bnpool_fwd_pairs): 152.4 / 136.4 / 149.0 us -- the 2x2 block needs 164 VGPRs
  // (3 waves / SIMD), the pair 94 (5 waves)
  const char* env = getenv("PDE_BNPOOL_FWD");
  const int variant = env ? atoi(env) : 2;
  if (variant == 2 || variant == 4) {
    const int jw = variant / 2, cells = (OW + jw - 1) / jw * CP;
    const int threads = min(256, (cells + 63) / 64 * 64);
    auto kern = jw == 2 ? k_bnpool_fwd2<2> : k_bnpool_fwd2<1>;
    hipLaunchKernelGGL(kern, dim3((OH + 1) / 2, N), dim3(threads), 0, st, (const uint4*)y, scale, shift, (uint4*)p,
                       (uint2*)arg, (uint4*)ysel, H, W, OH, OW, CP, ilog2(CP));
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_bnpool_fwd, dim3(OH, N), dim3(bnpool_threads(OW * CP)), 0, st, (const uint4*)y, scale, shift,
                     (uint4*)p, (uint2*)arg, (uint4*)ysel, H, W, OH, OW, CP, ilog2(CP));
  return hipGetLastError();
}

// part: pde_bnpool_part_floats(N, H, W, C) floats; coef: 3C floats.  The apply pass runs one thread per
// (column, chunk) of a pooled row: OW * C / 8 <= 512 (ResNet stem: 56 * 8 = 448).
hipError_t pde_bnpool_bwd(const void* dp, const void* arg, const void* y, const void* ysel, const float* scale,
                          const float* shift, const void* gamma, const float* mean, const float* rstd, float* part,
                          float* coef, void* dgamma, void* dbeta, void* dy, int N, int C, int H, int W, int OH, int OW,
                          hipStream_t st) {
  const int CP = C / 8;
  if (C % 8 || (CP & (CP - 1)) || CP > 64 || OW * CP > 512) return hipErrorInvalidValue;
  // column blocks of <= 256 threads (one per (column, chunk)) with one halo column each
  const int ncb = (OW * CP + 255) / 256, cols_per = (OW + ncb - 1) / ncb;
  const int lg = ilog2(CP), nt = (cols_per * CP + 63) / 64 * 64, gx = (OH + kBnpoolRB - 1) / kBnpoolRB;
  const size_t lds = (size_t)(kBnpoolRB + 1) * (cols_per + 1) * CP * 24;   // staged gradient (16 B) + argmax (8 B)
  if (lds > 65536 || nt > 256) return hipErrorInvalidValue;
  // BN partials from the pooled maps: rows = pooled cells, x = y[argmax], mask x*scale + shift > 0
  const int Mp = N * OH * OW, RP = 256 / CP;
  int nblk = pde_bn_blocks(Mp, C);
  hipLaunchKernelGGL(k_bn_bwd_reduce<2>, dim3(nblk), dim3(256), (size_t)RP * 2 * C * sizeof(float), st,
                     (const uint4*)dp, (const uint4*)nullptr, (const uint4*)ysel, mean, rstd, scale, shift, Mp, C,
                     (Mp + nblk - 1) / nblk, part, (uint4*)nullptr);
  float* pp = part;
  if (nblk > kFoldThreshold) {
    float* folded = part + (size_t)nblk * 2 * C;
    hipLaunchKernelGGL(k_fold_rows, dim3((2 * C + 255) / 256, kFoldRows), dim3(256), 0, st, part, nblk, 2 * C,
                       (nblk + kFoldRows - 1) / kFoldRows, folded);
    pp = folded;
    nblk = kFoldRows;
  }
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 63) / 64), dim3(1024), 0, st, pp, nblk, C, N * H * W,
                     (const bf16_t*)gamma, mean, rstd, (bf16_t*)dgamma, (bf16_t*)dbeta, coef);
  hipLaunchKernelGGL((k_bnpool_bwd<kBnpoolRB>), dim3(gx, N, ncb), dim3(nt), lds, st, (const uint4*)dp,
                     (const uint2*)arg, (const uint4*)y, scale, shift, (const float*)coef, (uint4*)dy, H, W, OH, OW,
                     CP, lg, cols_per);
  return hipGetLastError();
}

// relu with y == nullptr: the ReLU mask is recomputed from x with the forward's scale / shift (no
// residual in the forward), so y is not read
// pre_nblk > 0: `part` already holds [pre_nblk][2][C] reduction partials (summed by the dgrad epilogue
// that produced dy, conv.hip BnbArgs; relu == 2 semantics, no dres) and is sized
// pde_bn_part_rows(pre_nblk) x 2C: the reduce pass is skipped
hipError_t pde_bn_bwd(const void* dy, const void* y, const void* x, int M, int C, const void* gamma, const float* mean,
                      const float* rstd, const float* scale, const float* shift, float* part, float* coef,
                      void* dgamma, void* dbeta, void* dx, void* dres, int relu, int pre_nblk, hipStream_t st) {
  if (C % 8 != 0 || 256 % (C / 8) != 0) return hipErrorInvalidValue;
  if (relu && !y && (!scale || !shift)) return hipErrorInvalidValue;
  relu = !relu ? 0 : (y ? 1 : 2);
  if (pre_nblk > 0 && (relu != 2 || dres)) return hipErrorInvalidValue;
  const int CP = C / 8, RP = 256 / CP;
  int nblk = pre_nblk > 0 ? pre_nblk : pde_bn_blocks(M, C);
  const int rpb = (M + nblk - 1) / nblk;
  // ReLU after a residual add: the reduce pass writes the masked gradient as dres, and the apply pass
  // reads it back as its (unmasked) dy -- 7 tensor passes instead of 8 (the apply no longer reads dy
  // and y, and writes one tensor)
  const bool res_first = relu == 1 && dres;
  if (pre_nblk <= 0) {
    auto red = relu == 0 ? k_bn_bwd_reduce<0> : relu == 1 ? k_bn_bwd_reduce<1> : k_bn_bwd_reduce<2>;
    hipLaunchKernelGGL(red, dim3(nblk), dim3(256), (size_t)RP * 2 * C * sizeof(float), st, (const uint4*)dy,
                       (const uint4*)y, (const uint4*)x, mean, rstd, scale, shift, M, C, rpb, part,
                       res_first ? (uint4*)dres : (uint4*)nullptr);
  } else if (nblk > kFoldThreshold) {   // thousands of per-tile rows: pre-fold as the forward does
    float* folded = part + (size_t)nblk * 2 * C;
    hipLaunchKernelGGL(k_fold_rows, dim3((2 * C + 255) / 256, kFoldRows), dim3(256), 0, st, part, nblk, 2 * C,
                       (nblk + kFoldRows - 1) / kFoldRows, folded);
    part = folded;
    nblk = kFoldRows;
  }
  hipLaunchKernelGGL(k_bn_bwd_finalize, dim3((C + 63) / 64), dim3(1024), 0, st, part, nblk, C, M,
                     (const bf16_t*)gamma, mean, rstd, (bf16_t*)dgamma, (bf16_t*)dbeta, coef);
  const int64_t n8 = (int64_t)M * CP;
  if (res_first) {
    hipLaunchKernelGGL(k_bn_bwd_apply<0>, dim3(grid_cap(n8, 4096)), dim3(256), 0, st, (const uint4*)dres,
                       (const uint4*)nullptr, (const uint4*)x, coef, scale, shift, (uint4*)dx, (uint4*)nullptr, n8, C);
    return hipGetLastError();
  }
  auto app = relu == 0 ? k_bn_bwd_apply<0> : relu == 1 ? k_bn_bwd_apply<1> : k_bn_bwd_apply<2>;
  hipLaunchKernelGGL(app, dim3(grid_cap(n8, 4096)), dim3(256), 0, st, (const uint4*)dy, (const uint4*)y,
                     (const uint4*)x, coef, scale, shift, (uint4*)dx, (uint4*)dres, n8, C);
  return hipGetLastError();
}

hipError_t pde_maxpool3s2_fwd(const void* x, void* y, void* arg, int N, int C, int H, int W, int OH, int OW,
                              hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * OH * OW * (C / 8);
  hipLaunchKernelGGL(k_maxpool3s2_fwd, dim3(grid_cap(total, 8192)), dim3(256), 0, st, (const uint4*)x, (uint4*)y,
                     (uint2*)arg, N, H, W, OH, OW, C / 8);
  return hipGetLastError();
}

hipError_t pde_maxpool3s2_bwd(const void* dy, const void* arg, void* dx, int N, int C, int H, int W, int OH, int OW,
                              hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * H * W * (C / 8);
  hipLaunchKernelGGL(k_maxpool3s2_bwd, dim3(grid_cap(total, 8192)), dim3(256), 0, st, (const uint4*)dy,
                     (const uint2*)arg, (uint4*)dx, N, H, W, OH, OW, C / 8);
  return hipGetLastError();
}

hipError_t pde_sgd_master(float* master, void* p16, const void* g16, float* buf, int64_t n, float lr, float momentum,
                          float wd, int nesterov, float grad_scale, const uint8_t* decay_blk, hipStream_t st) {
  const int64_t n4 = n / 4;
  hipLaunchKernelGGL(k_sgd_master, dim3(grid_cap(n4, 2048)), dim3(256), 0, st, master, (uint2*)p16,
                     (const uint2*)g16, (float4*)buf, n4, lr, momentum, wd, nesterov, grad_scale, decay_blk);
  return hipGetLastError();
}

hipError_t pde_avgpool_fwd(const void* x, void* out, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int total = N * (C / 8);
  hipLaunchKernelGGL(k_avgpool_fwd, dim3((total + 255) / 256), dim3(256), 0, st, (const uint4*)x, (uint4*)out, N, HW,
                     C / 8, 1.f / (float)HW);
  return hipGetLastError();
}

hipError_t pde_avgpool_bwd(const void* dout, void* dx, int N, int HW, int C, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  const int64_t total = (int64_t)N * HW * (C / 8);
  hipLaunchKernelGGL(k_avgpool_bwd, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, st, (const uint4*)dout,
                     (uint4*)dx, N, HW, C / 8, 1.f / (float)HW);
  return hipGetLastError();
}

}  // extern "C"
