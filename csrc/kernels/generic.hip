// Generic fp32 CDNA4 kernels behind ``ops`` (Linear / Conv2d / ReLU / MaxPool / log_softmax /
// cross_entropy) for models other than the fused toy CNN (e.g. the MLP config) and for the
// reference-compatible autograd path.
//
//   k_gemm        : C[z] = op(A[z]) @ op(B[z]) (+ beta*C) (+ bias per row or column) (ReLU), batched
//                   over blockIdx.z by element strides; 64x64 block tile, BK = 16, 4 waves each 32x32
//                   on v_mfma_f32_16x16x4_f32 (2x2 fragments), next K-tile prefetched into registers
//                   while the current one is multiplied from LDS.  Epilogue can also atomically add
//                   (batched weight gradients reduced over the batch in the same launch).
//   k_xent_*      : fused log_softmax + NLL (mean / sum / none) forward and backward, wave per row
//   k_logsm_*     : row-wise log_softmax forward / backward
//   k_relu_*      : ReLU forward / backward (float4 vectorised, grid-stride)
//   k_pool2_*     : 2x2 stride-2 max pool with argmax codes, forward / backward
//   k_im2col / k_col2im, k_bias_grad_nchw, k_colsum
#include "pde_hip.h"
#include "pde_bf16.h"
#include "pde_kernels.h"

namespace {

constexpr int BM = 64, BN = 64, BK = 16;

template <bool TA, bool TB>
__device__ __forceinline__ void gemm_load(const float* __restrict__ A, const float* __restrict__ B, int M, int N,
                                          int K, int lda, int ldb, int m0, int n0, int k0, int t, float ra[4],
                                          float rb[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = t + 256 * j;
    int m, k;
    if (!TA) { m = e >> 4; k = e & 15; }          // A[m][k], k contiguous
    else { k = e >> 6; m = e & 63; }              // A stored [k][m], m contiguous
    const int gm = m0 + m, gk = k0 + k;
    const bool ok = gm < M && gk < K;
    const size_t idx = TA ? (size_t)min(gk, K - 1) * lda + min(gm, M - 1) : (size_t)min(gm, M - 1) * lda + min(gk, K - 1);
    const float v = A[idx];
    ra[j] = ok ? v : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = t + 256 * j;
    int n, k;
    if (!TB) { k = e >> 6; n = e & 63; }          // B[k][n], n contiguous
    else { n = e >> 4; k = e & 15; }              // B stored [n][k], k contiguous
    const int gn = n0 + n, gk = k0 + k;
    const bool ok = gn < N && gk < K;
    const size_t idx = TB ? (size_t)min(gn, N - 1) * ldb + min(gk, K - 1) : (size_t)min(gk, K - 1) * ldb + min(gn, N - 1);
    const float v = B[idx];
    rb[j] = ok ? v : 0.f;
  }
}

template <bool TA, bool TB>
__device__ __forceinline__ void gemm_store_lds(float (*As)[BM + 4], float (*Bs)[BN + 4], int t, const float ra[4],
                                               const float rb[4]) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int e = t + 256 * j;
    if (!TA) As[e & 15][e >> 4] = ra[j];
    else As[e >> 6][e & 63] = ra[j];
    if (!TB) Bs[e >> 6][e & 63] = rb[j];
    else Bs[e & 15][e >> 4] = rb[j];
  }
}

struct GemmArgs {
  const float* A; const float* B; float* C; const float* bias;
  int M, N, K, lda, ldb, ldc;
  long long sA, sB, sC;        // batch strides (elements)
  float alpha, beta;
  int bias_mode;               // 0 none, 1 per column (n), 2 per row (m)
  int relu;                    // apply ReLU in the epilogue
  int atomic;                  // epilogue atomically adds alpha*acc into C (batched reductions)
};

template <bool TA, bool TB>
__global__ __launch_bounds__(256) void k_gemm(GemmArgs g) {
  __shared__ float As[2][BK][BM + 4];
  __shared__ float Bs[2][BK][BN + 4];
  const int t = threadIdx.x, l = t & 63, w = t >> 6, wm = w >> 1, wn = w & 1;
  const int m0 = blockIdx.y * BM, n0 = blockIdx.x * BN, z = blockIdx.z;
  const float* A = g.A + z * g.sA;
  const float* B = g.B + z * g.sB;
  float* C = g.C + z * g.sC;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  float ra[4], rb[4];
  gemm_load<TA, TB>(A, B, g.M, g.N, g.K, g.lda, g.ldb, m0, n0, 0, t, ra, rb);
  gemm_store_lds<TA, TB>(As[0], Bs[0], t, ra, rb);
  __syncthreads();
  const int nk = (g.K + BK - 1) / BK;
  for (int kt = 0; kt < nk; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < nk) gemm_load<TA, TB>(A, B, g.M, g.N, g.K, g.lda, g.ldb, m0, n0, (kt + 1) * BK, t, ra, rb);
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      const int kr = kk * 4 + (l >> 4);
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[cur][kr][wm * 32 + i * 16 + (l & 15)];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[cur][kr][wn * 32 + j * 16 + (l & 15)];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma16x16x4(a[i], b[j], acc[i][j]);
    }
    if (kt + 1 < nk) {
      gemm_store_lds<TA, TB>(As[cur ^ 1], Bs[cur ^ 1], t, ra, rb);
    }
    __syncthreads();
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = m0 + wm * 32 + i * 16 + (l >> 4) * 4 + r;
        const int col = n0 + wn * 32 + j * 16 + (l & 15);
        if (row < g.M && col < g.N) {
          float* cp = C + (size_t)row * g.ldc + col;
          float v = g.alpha * acc[i][j][r];
          if (g.atomic) {
            atomicAdd(cp, v);
          } else {
            if (g.beta != 0.f) v += g.beta * *cp;
            if (g.bias_mode == 1) v += g.bias[col];
            else if (g.bias_mode == 2) v += g.bias[row];
            if (g.relu) v = fmaxf(v, 0.f);
            *cp = v;
          }
        }
      }
}

// ---------------------------------------------------------------------------------------------
// cross entropy over logits [B][C] (= F.cross_entropy = nll(log_softmax)), wave per row
// logits of either dtype (fp32 or bf16: the bf16 ResNet head feeds its own output, no cast kernel)
__device__ __forceinline__ float ld_logit(const float* p, size_t i) { return p[i]; }
__device__ __forceinline__ float ld_logit(const bf16_t* p, size_t i) { return bf2f(p[i]); }
__device__ __forceinline__ void st_logit(float* p, size_t i, float v) { p[i] = v; }
__device__ __forceinline__ void st_logit(bf16_t* p, size_t i, float v) { p[i] = f2bf(v); }

template <typename T>
__global__ __launch_bounds__(256) void k_xent_fwd(const T* __restrict__ x, const long long* __restrict__ y, int B,
                                                  int C, float* __restrict__ row_loss, float* __restrict__ lse_out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= B) return;
  const size_t r0 = (size_t)row * C;
  float m = -INFINITY;
  for (int c = l; c < C; c += 64) m = fmaxf(m, ld_logit(x, r0 + c));
  m = wave_max(m);
  float s = 0.f;
  for (int c = l; c < C; c += 64) s += expf(ld_logit(x, r0 + c) - m);
  s = wave_sum(s);
  const float lse = m + logf(s);
  if (l == 0) {
    const int yy = (int)y[row];
    row_loss[row] = (yy >= 0 && yy < C) ? lse - ld_logit(x, r0 + yy) : 0.f;
    lse_out[row] = lse;
  }
}

// dx = (softmax(x) - onehot(y)) * scale_row  (scale = grad * (1/B for mean))
template <typename T>
__global__ __launch_bounds__(256) void k_xent_bwd(const T* __restrict__ x, const long long* __restrict__ y,
                                                  const float* __restrict__ lse, const float* __restrict__ gscale,
                                                  int per_row, float mul, int B, int C, T* __restrict__ dx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= B) return;
  const float g = (per_row ? gscale[row] : gscale[0]) * mul;
  const int yy = (int)y[row];
  const float L = lse[row];
  const size_t r0 = (size_t)row * C;
  for (int c = l; c < C; c += 64)
    st_logit(dx, r0 + c, (expf(ld_logit(x, r0 + c) - L) - (c == yy ? 1.f : 0.f)) * g);
}

__global__ __launch_bounds__(256) void k_logsm_fwd(const float* __restrict__ x, int B, int C, float* __restrict__ out) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= B) return;
  const float* xr = x + (size_t)row * C;
  float m = -INFINITY;
  for (int c = l; c < C; c += 64) m = fmaxf(m, xr[c]);
  m = wave_max(m);
  float s = 0.f;
  for (int c = l; c < C; c += 64) s += expf(xr[c] - m);
  s = wave_sum(s);
  const float ls = logf(s);
  for (int c = l; c < C; c += 64) out[(size_t)row * C + c] = xr[c] - m - ls;
}

// d x = g - exp(out) * sum(g)
__global__ __launch_bounds__(256) void k_logsm_bwd(const float* __restrict__ out, const float* __restrict__ g, int B,
                                                   int C, float* __restrict__ dx) {
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
  if (row >= B) return;
  float s = 0.f;
  for (int c = l; c < C; c += 64) s += g[(size_t)row * C + c];
  s = wave_sum(s);
  for (int c = l; c < C; c += 64) dx[(size_t)row * C + c] = g[(size_t)row * C + c] - expf(out[(size_t)row * C + c]) * s;
}

__global__ __launch_bounds__(256) void k_relu_fwd(const float* __restrict__ x, float* __restrict__ y, long long n) {
  const long long n4 = n / 4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 v = reinterpret_cast<const float4*>(x)[i];
    v.x = fmaxf(v.x, 0.f); v.y = fmaxf(v.y, 0.f); v.z = fmaxf(v.z, 0.f); v.w = fmaxf(v.w, 0.f);
    reinterpret_cast<float4*>(y)[i] = v;
  }
  for (long long i = n4 * 4 + (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    y[i] = fmaxf(x[i], 0.f);
}

__global__ __launch_bounds__(256) void k_relu_bwd(const float* __restrict__ y, const float* __restrict__ g,
                                                  float* __restrict__ dx, long long n) {
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
    dx[i] = y[i] > 0.f ? g[i] : 0.f;
}

// 2x2 / stride 2 max pool over [NC][H][W] planes; code = dy*2+dx of the first maximum
__global__ __launch_bounds__(256) void k_pool2_fwd(const float* __restrict__ x, int NC, int H, int W,
                                                   float* __restrict__ y, uint8_t* __restrict__ code) {
  const int OH = H / 2, OW = W / 2;
  const long long n = (long long)NC * OH * OW;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int ow = (int)(i % OW), oh = (int)((i / OW) % OH);
    const long long pl = i / ((long long)OH * OW);
    const float* p = x + pl * H * W + (2 * oh) * W + 2 * ow;
    float best = p[0]; int c = 0;
    if (p[1] > best || (p[1] != p[1])) { best = p[1]; c = 1; }
    if (p[W] > best || (p[W] != p[W])) { best = p[W]; c = 2; }
    if (p[W + 1] > best || (p[W + 1] != p[W + 1])) { best = p[W + 1]; c = 3; }
    y[i] = best;
    code[i] = (uint8_t)c;
  }
}

__global__ __launch_bounds__(256) void k_pool2_bwd(const float* __restrict__ g, const uint8_t* __restrict__ code, int NC,
                                                   int H, int W, float* __restrict__ dx) {
  const long long n = (long long)NC * H * W;
  const int OH = H / 2, OW = W / 2;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int xw = (int)(i % W), xh = (int)((i / W) % H);
    const long long pl = i / ((long long)H * W);
    const int oh = xh / 2, ow = xw / 2;
    float v = 0.f;
    if (oh < OH && ow < OW) {
      const long long o = pl * OH * OW + (long long)oh * OW + ow;
      v = (code[o] == (xh & 1) * 2 + (xw & 1)) ? g[o] : 0.f;
    }
    dx[i] = v;
  }
}

// im2col: x [B][C][H][W] -> col [B][C*KH*KW][OH*OW]
__global__ __launch_bounds__(256) void k_im2col(const float* __restrict__ x, int B, int C, int H, int W, int KH, int KW,
                                                int stride, int pad, int OH, int OW, float* __restrict__ col) {
  const long long P = (long long)OH * OW, R = (long long)C * KH * KW, n = B * R * P;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long p = i % P, r = (i / P) % R, b = i / (P * R);
    const int ow = (int)(p % OW), oh = (int)(p / OW);
    const int kw = (int)(r % KW), kh = (int)((r / KW) % KH), c = (int)(r / (KW * KH));
    const int ih = oh * stride - pad + kh, iw = ow * stride - pad + kw;
    col[i] = (ih >= 0 && ih < H && iw >= 0 && iw < W) ? x[((b * C + c) * H + ih) * (long long)W + iw] : 0.f;
  }
}

// col2im (gather form, no atomics): dx[b][c][ih][iw] = sum of the col entries that read it
__global__ __launch_bounds__(256) void k_col2im(const float* __restrict__ col, int B, int C, int H, int W, int KH,
                                                int KW, int stride, int pad, int OH, int OW, float* __restrict__ dx) {
  const long long n = (long long)B * C * H * W, P = (long long)OH * OW, R = (long long)C * KH * KW;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int iw = (int)(i % W), ih = (int)((i / W) % H), c = (int)((i / ((long long)W * H)) % C);
    const long long b = i / ((long long)C * H * W);
    float s = 0.f;
    for (int kh = 0; kh < KH; ++kh) {
      const int th = ih + pad - kh;
      if (th < 0 || th % stride) continue;
      const int oh = th / stride;
      if (oh >= OH) continue;
      for (int kw = 0; kw < KW; ++kw) {
        const int tw = iw + pad - kw;
        if (tw < 0 || tw % stride) continue;
        const int ow = tw / stride;
        if (ow >= OW) continue;
        s += col[(b * R + ((long long)c * KH + kh) * KW + kw) * P + (long long)oh * OW + ow];
      }
    }
    dx[i] = s;
  }
}

// db[o] = sum_{b,p} dy[b][o][p]   (one block per output channel)
__global__ __launch_bounds__(256) void k_bias_grad_nchw(const float* __restrict__ dy, int B, int O, long long P,
                                                        float* __restrict__ db) {
  __shared__ float sc[4];
  const int o = blockIdx.x;
  float s = 0.f;
  for (long long i = threadIdx.x; i < (long long)B * P; i += 256) {
    const long long b = i / P, p = i % P;
    s += dy[(b * O + o) * P + p];
  }
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) sc[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) db[o] = sc[0] + sc[1] + sc[2] + sc[3];
}

// column sums of a [M][N] matrix (linear bias grad); block = 64 columns x 4 row groups
__global__ __launch_bounds__(256) void k_colsum(const float* __restrict__ x, int M, int N, float* __restrict__ out) {
  __shared__ float red[4][64];
  const int col = blockIdx.x * 64 + (threadIdx.x & 63), w = threadIdx.x >> 6;
  float s = 0.f;
  if (col < N)
    for (int r = w; r < M; r += 4) s += x[(size_t)r * N + col];
  red[w][threadIdx.x & 63] = s;
  __syncthreads();
  if (w == 0 && col < N) out[col] = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// rows gather: out[i] = src[idx[i]] (row length in floats, multiple of 4)
__global__ __launch_bounds__(256) void k_gather_rows(const float* __restrict__ src, const long long* __restrict__ idx,
                                                     int n, int row4, float* __restrict__ out) {
  const long long tot = (long long)n * row4;
  for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < tot; i += (long long)gridDim.x * 256) {
    const long long r = i / row4, c = i % row4;
    reinterpret_cast<float4*>(out)[i] = reinterpret_cast<const float4*>(src)[idx[r] * row4 + c];
  }
}

inline int ew_grid(long long n) {
  long long b = (n + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 4096 ? 4096 : b));
}

}  // namespace

extern "C" {

hipError_t pde_gemm_f32(const float* A, const float* B, float* C, const float* bias, int M, int N, int K, int lda,
                        int ldb, int ldc, int transA, int transB, long long sA, long long sB, long long sC, int batch,
                        float alpha, float beta, int bias_mode, int relu, int atomic, hipStream_t st) {
  GemmArgs g{A, B, C, bias, M, N, K, lda, ldb, ldc, sA, sB, sC, alpha, beta, bias_mode, relu, atomic};
  dim3 grid((N + BN - 1) / BN, (M + BM - 1) / BM, batch);
  if (!transA && !transB) hipLaunchKernelGGL((k_gemm<false, false>), grid, dim3(256), 0, st, g);
  else if (!transA && transB) hipLaunchKernelGGL((k_gemm<false, true>), grid, dim3(256), 0, st, g);
  else if (transA && !transB) hipLaunchKernelGGL((k_gemm<true, false>), grid, dim3(256), 0, st, g);
  else hipLaunchKernelGGL((k_gemm<true, true>), grid, dim3(256), 0, st, g);
  return hipGetLastError();
}

hipError_t pde_xent_fwd(const float* x, const long long* y, int B, int C, float* row_loss, float* lse,
                        hipStream_t st) {
  hipLaunchKernelGGL(k_xent_fwd<float>, dim3((B + 3) / 4), dim3(256), 0, st, x, y, B, C, row_loss, lse);
  return hipGetLastError();
}

hipError_t pde_xent_bwd(const float* x, const long long* y, const float* lse, const float* gscale, int per_row,
                        float mul, int B, int C, float* dx, hipStream_t st) {
  hipLaunchKernelGGL(k_xent_bwd<float>, dim3((B + 3) / 4), dim3(256), 0, st, x, y, lse, gscale, per_row, mul, B, C, dx);
  return hipGetLastError();
}

hipError_t pde_xent_fwd_bf16(const void* x, const long long* y, int B, int C, float* row_loss, float* lse,
                             hipStream_t st) {
  hipLaunchKernelGGL(k_xent_fwd<bf16_t>, dim3((B + 3) / 4), dim3(256), 0, st, (const bf16_t*)x, y, B, C, row_loss,
                     lse);
  return hipGetLastError();
}

hipError_t pde_xent_bwd_bf16(const void* x, const long long* y, const float* lse, const float* gscale, int per_row,
                             float mul, int B, int C, void* dx, hipStream_t st) {
  hipLaunchKernelGGL(k_xent_bwd<bf16_t>, dim3((B + 3) / 4), dim3(256), 0, st, (const bf16_t*)x, y, lse, gscale,
                     per_row, mul, B, C, (bf16_t*)dx);
  return hipGetLastError();
}

hipError_t pde_log_softmax_fwd(const float* x, int B, int C, float* out, hipStream_t st) {
  hipLaunchKernelGGL(k_logsm_fwd, dim3((B + 3) / 4), dim3(256), 0, st, x, B, C, out);
  return hipGetLastError();
}

hipError_t pde_log_softmax_bwd(const float* out, const float* g, int B, int C, float* dx, hipStream_t st) {
  hipLaunchKernelGGL(k_logsm_bwd, dim3((B + 3) / 4), dim3(256), 0, st, out, g, B, C, dx);
  return hipGetLastError();
}

hipError_t pde_relu_fwd(const float* x, float* y, long long n, hipStream_t st) {
  hipLaunchKernelGGL(k_relu_fwd, dim3(ew_grid((n + 3) / 4)), dim3(256), 0, st, x, y, n);
  return hipGetLastError();
}

hipError_t pde_relu_bwd(const float* y, const float* g, float* dx, long long n, hipStream_t st) {
  hipLaunchKernelGGL(k_relu_bwd, dim3(ew_grid(n)), dim3(256), 0, st, y, g, dx, n);
  return hipGetLastError();
}

hipError_t pde_pool2_fwd(const float* x, int NC, int H, int W, float* y, uint8_t* code, hipStream_t st) {
  hipLaunchKernelGGL(k_pool2_fwd, dim3(ew_grid((long long)NC * (H / 2) * (W / 2))), dim3(256), 0, st, x, NC, H, W, y,
                     code);
  return hipGetLastError();
}

hipError_t pde_pool2_bwd(const float* g, const uint8_t* code, int NC, int H, int W, float* dx, hipStream_t st) {
  hipLaunchKernelGGL(k_pool2_bwd, dim3(ew_grid((long long)NC * H * W)), dim3(256), 0, st, g, code, NC, H, W, dx);
  return hipGetLastError();
}

hipError_t pde_im2col(const float* x, int B, int C, int H, int W, int KH, int KW, int stride, int pad, int OH, int OW,
                      float* col, hipStream_t st) {
  const long long n = (long long)B * C * KH * KW * OH * OW;
  hipLaunchKernelGGL(k_im2col, dim3(ew_grid(n)), dim3(256), 0, st, x, B, C, H, W, KH, KW, stride, pad, OH, OW, col);
  return hipGetLastError();
}

hipError_t pde_col2im(const float* col, int B, int C, int H, int W, int KH, int KW, int stride, int pad, int OH,
                      int OW, float* dx, hipStream_t st) {
  const long long n = (long long)B * C * H * W;
  hipLaunchKernelGGL(k_col2im, dim3(ew_grid(n)), dim3(256), 0, st, col, B, C, H, W, KH, KW, stride, pad, OH, OW, dx);
  return hipGetLastError();
}

hipError_t pde_bias_grad_nchw(const float* dy, int B, int O, long long P, float* db, hipStream_t st) {
  hipLaunchKernelGGL(k_bias_grad_nchw, dim3(O), dim3(256), 0, st, dy, B, O, P, db);
  return hipGetLastError();
}

hipError_t pde_colsum(const float* x, int M, int N, float* out, hipStream_t st) {
  hipLaunchKernelGGL(k_colsum, dim3((N + 63) / 64), dim3(256), 0, st, x, M, N, out);
  return hipGetLastError();
}

hipError_t pde_gather_rows(const float* src, const long long* idx, int n, int row_floats, float* out, hipStream_t st) {
  if (row_floats % 4) return hipErrorInvalidValue;
  const int row4 = row_floats / 4;
  hipLaunchKernelGGL(k_gather_rows, dim3(ew_grid((long long)n * row4)), dim3(256), 0, st, src, idx, n, row4, out);
  return hipGetLastError();
}

}  // extern "C"
