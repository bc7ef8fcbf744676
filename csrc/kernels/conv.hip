// Implicit-GEMM convolutions on bf16 MFMA (gfx950) for the ResNet-18 config of BASELINE.json
// ("ResNet-18 bf16 ... MFMA conv-as-GEMM path").  Activations are NHWC (channels-last) bf16, weights
// are torch's channels-last [Cout][R][S][Cin] (= [N][tap][C]), accumulation is fp32.
//
// Three GEMM views of one convolution (stride s, pad p, taps t = (r, q)):
//   fprop : Y[m=(b,oh,ow)][n]  = sum_{t,c} X[b, oh*s-p+r, ow*s-p+q][c] * W[n][t][c]
//   dgrad : dX[m=(b,h,w)][c]   = sum_{t,n} dY[b, (h+p-r)/s, (w+p-q)/s][n] * W[n][t][c]
//           (only taps with (h+p-r) % s == 0 contribute: the output pixels are split into s*s
//           phases (h%s, w%s), each a dense implicit GEMM over its own tap subset -- no masked MFMA
//           work; a phase without taps (1x1 / stride 2) just writes zeros)
//   wgrad : dW[n][t][c]         = sum_{m=(b,oh,ow)} dY[m][n] * X[b, oh*s-p+r, ow*s-p+q][c]
// fprop and dgrad share one kernel (k_igemm): the A operand is a per-tap gather of 8-channel (16 B)
// vectors of an NHWC tensor, zero outside the image; the B operand is a weight matrix whose rows
// are K-contiguous (dgrad uses the transposed weights Wt[c][t][n], made by k_wtrans).
//
// Tiles (k_igemm): 256 threads = 4 waves, block tile BM x BN (256x64 or 128x128), K staged 64 deep;
// every wave owns a 64x64 sub-tile = 2x2 v_mfma_f32_32x32x16_bf16 accumulators.  Each stage is one
// (tap, 64-channel) slice: its A image [BM][64] and B image [BN][64] live in LDS as XOR-swizzled
// 128-byte rows (cdna_hip_programming.md T10 layout (a): conflict-free ds_read_b128 for the 32x32x16
// row operands).  Stages are double buffered: the global loads of stage k+1 are issued before the
// MFMAs of stage k and written to the other buffer after them; one barrier per stage.
// Epilogue: the fp32 accumulators are rounded to bf16 into an LDS tile and stored as coalesced 16 B
// rows; fprop can also emit per-channel (sum, sum of squares) partials of the rounded output in the
// [mtile][2][C] format of the BatchNorm finalize kernel (resnet.hip), so BN needs no stats pass.
//
// wgrad (k_wgrad): the reduction runs over pixels, which are the ROW index of both stored operands,
// so both fragments are hardware-transposed reads (ds_read_b64_tr_b16) of [64 pixel][64 ch] images;
// the pixel range is split across blocks (split-K) into fp32 slabs [split][N][T*C] that
// k_wgrad_reduce sums into the bf16 gradient.
#include "pde_hip.h"
#include "pde_bf16.h"
#include "pde_kernels.h"

namespace {

typedef short s4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) s4v lds_s4v;

// Bounds-checked buffer loads: an offset past the resource's size returns zeros, so image padding
// and ragged tiles cost no branch around the load (cdna_hip_programming.md T8 / §5.5 trap (c)).
typedef __amdgpu_buffer_rsrc_t rsrc_t;
constexpr uint32_t kOOB = 0x80000000u;
__device__ __forceinline__ rsrc_t make_rsrc(const void* p, uint32_t bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ uint4 bload16(rsrc_t r, uint32_t off) {
  return __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}

__device__ __forceinline__ f32x16 mfma_bf16(bf16x8 a, bf16x8 b, f32x16 c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

// byte offset of 16-byte chunk `ch` (0..7) of row `row` in a [rows][64 bf16] image
__device__ __forceinline__ int toff(int row, int ch) {
  return 1024 * (row >> 3) + 512 * (ch >> 2) + 64 * (row & 7) + 16 * ((ch & 3) ^ ((row >> 2) & 3));
}
__device__ __forceinline__ bf16x8 row_frag(const char* img, int row, int ch) {
  return *reinterpret_cast<const bf16x8*>(img + toff(row, ch));
}
// transposed operand of a 16-row k-step: lane (r = l&31, h = l>>5) gets column col0 + r of rows
// row0 + {4h..4h+3, 8+4h..8+4h+3}.  EXEC must be full.
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int row0, int col0) {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = (col0 >> 3) + 2 * (g & 1) + (p >> 1);
  const int r = row0 + 4 * h + q;
  const s4v v0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(img + toff(r, ch) + 8 * (p & 1)));
  const s4v v1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_s4v*)(img + toff(r + 8, ch) + 8 * (p & 1)));
  bf16x8 out;
  out[0] = v0[0]; out[1] = v0[1]; out[2] = v0[2]; out[3] = v0[3];
  out[4] = v1[0]; out[5] = v1[1]; out[6] = v1[2]; out[7] = v1[3];
  return out;
}

// ============================================================================ fprop / dgrad
struct Phase {
  int ph, pw, Hq, Wq, ntap;
  signed char dh[9], dw[9], widx[9];
};
struct IgemmArgs {
  const bf16_t* A;      // gather source NHWC [Bn][IH][IW][CA]
  const bf16_t* W;      // [NC][T][CA]
  bf16_t* Y;            // NHWC [Bn][OH][OW][NC]
  float* stats;         // optional [mtiles][2][NC] (single-phase launches)
  uint32_t a_bytes, w_bytes;
  int Bn, IH, IW, CA;
  int OH, OW, NC, T;
  int sA, sO;           // source pixel = q * sA + d ; output pixel = q * sO + phase offset
  int nphase, mtiles, ntiles;
  Phase phase[4];
};

constexpr int kThreads = 256;

template <int BM, int BN>
__global__ __launch_bounds__(kThreads, 2) void k_igemm(IgemmArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  static_assert(WM * 64 == BM, "wave grid must tile BM x BN with 64x64 wave tiles");
  constexpr int AU = BM / 32, BU = BN / 32;         // 16-B chunks per thread per stage
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, STAGE = ABYTES + BBYTES;
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  const int per_phase = a.mtiles * a.ntiles;
  const int phz = id / per_phase, rem = id % per_phase;
  const int mt = rem / a.ntiles, nt = rem % a.ntiles;
  const Phase& P = a.phase[phz];
  const int Mq = a.Bn * P.Hq * P.Wq;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= Mq) return;                              // whole block (phase grids differ in size)
  const int CPT = a.CA >> 6;                         // 64-channel stages per tap
  const int KT = P.ntap * CPT;
  const int ldw = a.T * a.CA;

  // ---- per-thread gather rows (fixed for the whole K loop) ----
  const int ch = t & 7;
  int pix[AU], hb[AU], wb[AU];
#pragma unroll
  for (int u = 0; u < AU; ++u) {
    const int m = m0 + (t >> 3) + 32 * u;
    if (m < Mq) {
      const int b = m / (P.Hq * P.Wq), r2 = m % (P.Hq * P.Wq);
      const int hq = r2 / P.Wq, wq = r2 % P.Wq;
      pix[u] = b * a.IH * a.IW;
      hb[u] = hq * a.sA;
      wb[u] = wq * a.sA;
    } else {
      pix[u] = 0;
      hb[u] = -(1 << 20);                             // always out of the image -> zeros
      wb[u] = 0;
    }
  }
  const rsrc_t ar = make_rsrc(a.A, a.a_bytes), wr = make_rsrc(a.W, a.w_bytes);
  uint32_t wrow[BU];
#pragma unroll
  for (int v = 0; v < BU; ++v) wrow[v] = ((n0 + (t >> 3) + 32 * v) * ldw + ch * 8) * 2;

  uint4 ra[AU], rb[BU];
  auto load_stage = [&](int kt) {
    const int tap = kt / CPT, c0 = (kt - tap * CPT) * 64;
    const int dh = P.dh[tap], dw = P.dw[tap], wi = P.widx[tap];
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int ih = hb[u] + dh, iw = wb[u] + dw;
      const bool ok = (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const uint32_t off = ((uint32_t)((pix[u] + ih * a.IW + iw) * a.CA + c0 + ch * 8)) * 2u;
      ra[u] = bload16(ar, ok ? off : kOOB);
    }
#pragma unroll
    for (int v = 0; v < BU; ++v) rb[v] = bload16(wr, wrow[v] + (uint32_t)(wi * a.CA + c0) * 2u);
  };
  auto store_stage = [&](int buf) {
    char* Ai = smem + buf * STAGE;
    char* Bi = Ai + ABYTES;
#pragma unroll
    for (int u = 0; u < AU; ++u) *reinterpret_cast<uint4*>(Ai + toff((t >> 3) + 32 * u, ch)) = ra[u];
#pragma unroll
    for (int v = 0; v < BU; ++v) *reinterpret_cast<uint4*>(Bi + toff((t >> 3) + 32 * v, ch)) = rb[v];
  };

  const int wm = w / WN, wn = w % WN, lr = l & 31, lh = l >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0.f};

  if (KT > 0) {
    load_stage(0);
    store_stage(0);
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
      const bool more = kt + 1 < KT;
      if (more) load_stage(kt + 1);
      const char* Ai = smem + (kt & 1) * STAGE;
      const char* Bi = Ai + ABYTES;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) fa[i] = row_frag(Ai, wm * 64 + i * 32 + lr, 2 * s + lh);
#pragma unroll
        for (int j = 0; j < 2; ++j) fb[j] = row_frag(Bi, wn * 64 + j * 32 + lr, 2 * s + lh);
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
      }
      if (more) store_stage((kt + 1) & 1);
      __syncthreads();
    }
  }

  // ---- epilogue: bf16 tile through LDS, coalesced NHWC rows; optional BN partial stats ----
  constexpr int RS = BN * 2 + 16;                    // padded LDS row stride (bytes)
  static_assert(BM * RS + 2 * WM * BN * 4 <= 2 * STAGE, "epilogue LDS");
  char* ot = smem;
  float* sst = reinterpret_cast<float*>(smem + BM * RS);   // [WM][2][BN]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = wn * 64 + j * 32 + lr;
      float s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = wm * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
        const bf16_t hv = f2bf(acc[i][j][q]);
        *reinterpret_cast<bf16_t*>(ot + m * RS + n * 2) = hv;
        const float fv = bf2f(hv);
        s1 += fv;
        s2 += fv * fv;
      }
      if (a.stats) {
        s1 += __shfl_xor(s1, 32, 64);
        s2 += __shfl_xor(s2, 32, 64);
        if (i == 0) {
          if (lh == 0) { sst[(wm * 2 + 0) * BN + n] = s1; sst[(wm * 2 + 1) * BN + n] = s2; }
        } else {
          if (lh == 0) { sst[(wm * 2 + 0) * BN + n] += s1; sst[(wm * 2 + 1) * BN + n] += s2; }
        }
      }
    }
  __syncthreads();
  constexpr int CPR = BN / 8;                        // 16-B chunks per output row
#pragma unroll
  for (int u = 0; u < BM * CPR / kThreads; ++u) {
    const int c = t + kThreads * u, row = c / CPR, cc = c % CPR;
    const int m = m0 + row;
    if (m < Mq) {
      const int b = m / (P.Hq * P.Wq), r2 = m % (P.Hq * P.Wq);
      const int oh = (r2 / P.Wq) * a.sO + P.ph, ow = (r2 % P.Wq) * a.sO + P.pw;
      const uint4 v = *reinterpret_cast<const uint4*>(ot + row * RS + cc * 16);
      *reinterpret_cast<uint4*>(a.Y + (((size_t)b * a.OH + oh) * a.OW + ow) * a.NC + n0 + cc * 8) = v;
    }
  }
  if (a.stats && t < 2 * BN) {
    const int which = t / BN, n = t % BN;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WM; ++k) s += sst[(k * 2 + which) * BN + n];
    a.stats[((size_t)mt * 2 + which) * a.NC + n0 + n] = s;
  }
}

// Wt[c][t][n] = W[n][t][c]  (64x64 tiles through LDS; grid (C/64, N/64, T))
__global__ __launch_bounds__(256) void k_wtrans(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wt, int N,
                                                int T, int C) {
  __shared__ bf16_t sh[64][66];
  const int c0 = blockIdx.x * 64, n0 = blockIdx.y * 64, tap = blockIdx.z, t = threadIdx.x;
  for (int e = t; e < 64 * 64; e += 256) {
    const int n = e >> 6, c = e & 63;
    sh[n][c] = W[((size_t)(n0 + n) * T + tap) * C + c0 + c];
  }
  __syncthreads();
  for (int e = t; e < 64 * 64; e += 256) {
    const int c = e >> 6, n = e & 63;
    Wt[((size_t)(c0 + c) * T + tap) * N + n0 + n] = sh[n][c];
  }
}

// ============================================================================ wgrad
struct WgradArgs {
  const bf16_t* dY;     // [P][N]
  const bf16_t* X;      // [Bn][IH][IW][C]
  float* part;          // [splits][N][T*C]
  uint32_t dy_bytes, x_bytes;
  int Bn, IH, IW, C, OH, OW, N, S, stride, pad, T;
  int P, stages_per_split, mtiles, ntiles;
};

template <int BM, int BN>
__global__ __launch_bounds__(kThreads, 2) void k_wgrad(WgradArgs a) {
  constexpr int WN = (BN / 64 >= 4) ? 4 : BN / 64;   // waves along the (tap, c) columns
  constexpr int WM = 4 / WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM * WN == 4, "wgrad tiling");
  constexpr int AI = BM / 64, BI = BN / 64;          // 64-column images per operand
  constexpr int ABYTES = AI * 8192, BBYTES = BI * 8192, STAGE = ABYTES + BBYTES;
  constexpr int AU = BM / 32, BU = BN / 32;          // 16-B chunks per thread per stage (64 rows)
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int t = threadIdx.x, l = t & 63, w = t >> 6;
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = a.mtiles * a.ntiles;
  const int split = id / ntile, rem = id % ntile;
  const int mt = rem / a.ntiles, nt = rem % a.ntiles;
  const int n0 = mt * BM, k0 = nt * BN;              // output rows (Cout) / columns (tap, c)
  const int TC = a.T * a.C;
  const int pbeg = split * a.stages_per_split * 64;
  const int pend = min(a.P, pbeg + a.stages_per_split * 64);
  const int KT = (pend - pbeg + 63) / 64;

  // chunk -> (pixel row, column chunk): dY rows hold BM/8 chunks, X rows BN/8 chunks
  constexpr int ACPR = BM / 8, BCPR = BN / 8;
  int xtap_r[BU], xtap_s[BU], xc[BU];
  bool xcol_ok[BU];
#pragma unroll
  for (int v = 0; v < BU; ++v) {
    const int c = t + kThreads * v, cc = c % BCPR;
    const int col = k0 + cc * 8;
    xcol_ok[v] = col < TC;
    const int tap = min(col, TC - 1) / a.C;
    xc[v] = min(col, TC - 1) - tap * a.C;
    xtap_r[v] = tap / a.S - a.pad;
    xtap_s[v] = tap % a.S - a.pad;
  }
  const rsrc_t dyr = make_rsrc(a.dY, a.dy_bytes), xr = make_rsrc(a.X, a.x_bytes);
  uint4 ra[AU], rb[BU];
  auto load_stage = [&](int kt) {
    const int p0 = pbeg + kt * 64;
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int c = t + kThreads * u, row = c / ACPR, cc = c % ACPR;
      const int p = p0 + row;
      ra[u] = bload16(dyr, p < pend ? (uint32_t)(p * a.N + n0 + cc * 8) * 2u : kOOB);
    }
#pragma unroll
    for (int v = 0; v < BU; ++v) {
      const int c = t + kThreads * v, row = c / BCPR;
      const int p = p0 + row;
      bool ok = p < pend && xcol_ok[v];
      const int pp = min(p, a.P - 1);
      const int b = pp / (a.OH * a.OW), r2 = pp % (a.OH * a.OW);
      const int ih = (r2 / a.OW) * a.stride + xtap_r[v], iw = (r2 % a.OW) * a.stride + xtap_s[v];
      ok = ok && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const uint32_t off = (uint32_t)(((b * a.IH + ih) * a.IW + iw) * a.C + xc[v]) * 2u;
      rb[v] = bload16(xr, ok ? off : kOOB);
    }
  };
  auto store_stage = [&](int buf) {
    char* Ai = smem + buf * STAGE;
    char* Bi = Ai + ABYTES;
#pragma unroll
    for (int u = 0; u < AU; ++u) {
      const int c = t + kThreads * u, row = c / ACPR, cc = c % ACPR;
      *reinterpret_cast<uint4*>(Ai + (cc >> 3) * 8192 + toff(row, cc & 7)) = ra[u];
    }
#pragma unroll
    for (int v = 0; v < BU; ++v) {
      const int c = t + kThreads * v, row = c / BCPR, cc = c % BCPR;
      *reinterpret_cast<uint4*>(Bi + (cc >> 3) * 8192 + toff(row, cc & 7)) = rb[v];
    }
  };

  const int wm = w / WN, wn = w % WN, lr = l & 31;
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{0.f};

  if (KT > 0) {
    load_stage(0);
    store_stage(0);
    __syncthreads();
    for (int kt = 0; kt < KT; ++kt) {
      const bool more = kt + 1 < KT;
      if (more) load_stage(kt + 1);
      const char* Ai = smem + (kt & 1) * STAGE;
      const char* Bi = Ai + ABYTES;
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        bf16x8 fa[TM], fb[TN];
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int col = wm * (BM / WM) + i * 32;
          fa[i] = tr_frag(Ai + (col >> 6) * 8192, 16 * s, col & 63);
        }
#pragma unroll
        for (int j = 0; j < TN; ++j) {
          const int col = wn * (BN / WN) + j * 32;
          fb[j] = tr_frag(Bi + (col >> 6) * 8192, 16 * s, col & 63);
        }
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
      }
      if (more) store_stage((kt + 1) & 1);
      __syncthreads();
    }
  }
  // D[n][k']: lane column k' = col + lr, registers = rows n
  float* out = a.part + (size_t)split * a.N * TC;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int col = k0 + wn * (BN / WN) + j * 32 + lr;
      if (col < TC) {
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int n = n0 + wm * (BM / WM) + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * (l >> 5);
          out[(size_t)n * TC + col] = acc[i][j][q];
        }
      }
    }
}

// dW (bf16) = sum over splits of the fp32 slabs; 4 elements per thread
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ part, int splits, int64_t n,
                                                      bf16_t* __restrict__ dw) {
  const int64_t i = (blockIdx.x * 256ll + threadIdx.x) * 4;
  if (i >= n) return;
  float4 s = *reinterpret_cast<const float4*>(part + i);
  for (int k = 1; k < splits; ++k) {
    const float4 v = *reinterpret_cast<const float4*>(part + (size_t)k * n + i);
    s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
  }
  const float f[4] = {s.x, s.y, s.z, s.w};
  *reinterpret_cast<uint2*>(dw + i) = pack4(f);
}

template <int BM, int BN>
hipError_t launch_igemm(IgemmArgs& a, hipStream_t st) {
  int maxm = 0;
  for (int z = 0; z < a.nphase; ++z) maxm = max(maxm, a.Bn * a.phase[z].Hq * a.phase[z].Wq);
  a.mtiles = (maxm + BM - 1) / BM;
  a.ntiles = a.NC / BN;
  const int grid = a.nphase * a.mtiles * a.ntiles;
  hipLaunchKernelGGL((k_igemm<BM, BN>), dim3(grid), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t dispatch_igemm(IgemmArgs& a, hipStream_t st) {
  if (a.NC % 128 == 0) return launch_igemm<128, 128>(a, st);
  return launch_igemm<256, 64>(a, st);
}

}  // namespace

extern "C" {

int pde_conv_fprop_mtiles(int M, int N) { return N % 128 == 0 ? (M + 127) / 128 : (M + 255) / 256; }

hipError_t pde_conv_fprop(const void* x, const void* w, void* y, float* stats, int Bn, int H, int W, int C, int N,
                          int R, int S, int stride, int pad, int OH, int OW, hipStream_t st) {
  if (C % 64 || N % 64 || R * S > 9) return hipErrorInvalidValue;
  IgemmArgs a{};
  a.A = (const bf16_t*)x;
  a.W = (const bf16_t*)w;
  a.Y = (bf16_t*)y;
  a.stats = stats;
  a.a_bytes = (uint32_t)((size_t)Bn * H * W * C * 2);
  a.w_bytes = (uint32_t)((size_t)N * R * S * C * 2);
  a.Bn = Bn; a.IH = H; a.IW = W; a.CA = C;
  a.OH = OH; a.OW = OW; a.NC = N; a.T = R * S;
  a.sA = stride; a.sO = 1; a.nphase = 1;
  Phase& P = a.phase[0];
  P.ph = P.pw = 0; P.Hq = OH; P.Wq = OW; P.ntap = R * S;
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < S; ++s) {
      const int k = r * S + s;
      P.dh[k] = (signed char)(r - pad);
      P.dw[k] = (signed char)(s - pad);
      P.widx[k] = (signed char)k;
    }
  return dispatch_igemm(a, st);
}

hipError_t pde_conv_wtrans(const void* w, void* wt, int N, int T, int C, hipStream_t st) {
  if (N % 64 || C % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wtrans, dim3(C / 64, N / 64, T), dim3(256), 0, st, (const bf16_t*)w, (bf16_t*)wt, N, T, C);
  return hipGetLastError();
}

// dX (NHWC [Bn][H][W][C]) from dY ([Bn][OH][OW][N]) and Wt = [C][R*S][N] (pde_conv_wtrans)
hipError_t pde_conv_dgrad(const void* dy, const void* wt, void* dx, int Bn, int H, int W, int C, int N, int R, int S,
                          int stride, int pad, int OH, int OW, hipStream_t st) {
  if (C % 64 || N % 64 || R * S > 9 || stride < 1 || stride > 2) return hipErrorInvalidValue;
  IgemmArgs a{};
  a.A = (const bf16_t*)dy;
  a.W = (const bf16_t*)wt;
  a.Y = (bf16_t*)dx;
  a.stats = nullptr;
  a.a_bytes = (uint32_t)((size_t)Bn * OH * OW * N * 2);
  a.w_bytes = (uint32_t)((size_t)N * R * S * C * 2);
  a.Bn = Bn; a.IH = OH; a.IW = OW; a.CA = N;
  a.OH = H; a.OW = W; a.NC = C; a.T = R * S;
  a.sA = 1; a.sO = stride; a.nphase = stride * stride;
  for (int z = 0; z < a.nphase; ++z) {
    Phase& P = a.phase[z];
    P.ph = z / stride; P.pw = z % stride;
    P.Hq = (H - P.ph + stride - 1) / stride;
    P.Wq = (W - P.pw + stride - 1) / stride;
    P.ntap = 0;
    for (int r = 0; r < R; ++r) {
      const int nh = P.ph + pad - r;
      if (((nh % stride) + stride) % stride) continue;
      for (int s = 0; s < S; ++s) {
        const int nw = P.pw + pad - s;
        if (((nw % stride) + stride) % stride) continue;
        const int k = P.ntap++;
        // floor division of (possibly negative) exact multiples of stride
        P.dh[k] = (signed char)(nh >= 0 ? nh / stride : -((-nh) / stride));
        P.dw[k] = (signed char)(nw >= 0 ? nw / stride : -((-nw) / stride));
        P.widx[k] = (signed char)(r * S + s);
      }
    }
  }
  return dispatch_igemm(a, st);
}

int pde_conv_wgrad_splits(int Bn, int OH, int OW, int N, int T, int C) {
  // ~2 blocks per CU in total and >= 16 pixel stages per block: enough parallelism without
  // making the fp32 slab round trip (splits x N x T*C x 4 B, written and re-read) dominate.
  const int P = Bn * OH * OW, stages = (P + 63) / 64;
  const int BM = N % 128 == 0 ? 128 : 64, BN = 128;
  const int tiles = (N / BM) * ((T * C + BN - 1) / BN);
  int splits = (512 + tiles - 1) / tiles;
  splits = min(splits, stages / 16);
  return max(1, splits);
}

// part: fp32 [splits][N][T*C] scratch; dw: bf16 [N][T*C]
hipError_t pde_conv_wgrad(const void* dy, const void* x, float* part, int splits, void* dw, int Bn, int H, int W,
                          int C, int N, int R, int S, int stride, int pad, int OH, int OW, hipStream_t st) {
  if (C % 64 || N % 64 || splits < 1) return hipErrorInvalidValue;
  WgradArgs a{};
  a.dY = (const bf16_t*)dy;
  a.X = (const bf16_t*)x;
  a.part = part;
  a.dy_bytes = (uint32_t)((size_t)Bn * OH * OW * N * 2);
  a.x_bytes = (uint32_t)((size_t)Bn * H * W * C * 2);
  a.Bn = Bn; a.IH = H; a.IW = W; a.C = C; a.OH = OH; a.OW = OW; a.N = N; a.S = S;
  a.stride = stride; a.pad = pad; a.T = R * S;
  a.P = Bn * OH * OW;
  const int stages = (a.P + 63) / 64;
  a.stages_per_split = (stages + splits - 1) / splits;
  const int TC = a.T * C;
  if (N % 128 == 0) {
    a.mtiles = N / 128; a.ntiles = (TC + 127) / 128;
    hipLaunchKernelGGL((k_wgrad<128, 128>), dim3(splits * a.mtiles * a.ntiles), dim3(kThreads), 0, st, a);
  } else {
    a.mtiles = N / 64; a.ntiles = (TC + 127) / 128;
    hipLaunchKernelGGL((k_wgrad<64, 128>), dim3(splits * a.mtiles * a.ntiles), dim3(kThreads), 0, st, a);
  }
  PDE_HIP_CHECK(hipGetLastError());
  const int64_t n = (int64_t)N * TC;
  hipLaunchKernelGGL(k_wgrad_reduce, dim3((unsigned)((n / 4 + 255) / 256)), dim3(256), 0, st, part, splits, n,
                     (bf16_t*)dw);
  return hipGetLastError();
}

}  // extern "C"
