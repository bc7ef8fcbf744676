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
#include "pde_lds.h"

#include <cstdlib>

namespace {

using namespace pde_lds;

// p / d for 0 <= p < 2^23 via a float reciprocal and one correction step (no integer division in
// the K loop: its ~40-instruction expansion per row made wgrad VALU-bound)
__device__ __forceinline__ int fdiv(int p, int d, float inv) {
  int q = (int)((float)p * inv);
  const int r = p - q * d;
  q += r < 0 ? -1 : (r >= d ? 1 : 0);
  return q;
}

template <int S, int TM, int TN>
__device__ __forceinline__ void wg_frags(uint2 ab, uint2 bb, bf16x8* fa, bf16x8* fb) {
  static_assert(TM <= 2 && TN <= 2, "wg_frags: at most 2 x 2 fragments");
  fa[0] = trpair<2048 * S>(ab);
  if constexpr (TM > 1) fa[1] = trpair<2048 * S + colblk_off(1)>(ab);
  fb[0] = trpair<2048 * S>(bb);
  if constexpr (TN > 1) fb[1] = trpair<2048 * S + colblk_off(1)>(bb);
}

// ============================================================================ fprop / dgrad
struct Phase {
  int ph, pw, Hq, Wq, ntap;
  int ntap2;                     // 1: this phase also runs the second source's stages (below)
  float inv_hw, inv_w;           // 1 / (Hq * Wq), 1 / Wq for fdiv
  // per tap, packed into one dword so the wave-uniform lookup in the K loop is a scalar load
  // (byte-sized kernarg elements become VECTOR loads, whose vmcnt wait would drain the in-flight
  // LDS-DMA stages): bits 0-7 dh, 8-15 dw (signed), 16-23 weight tap index
  int tap[9];
};
__host__ __device__ inline int pack_tap(int dh, int dw, int widx) {
  return (dh & 0xff) | ((dw & 0xff) << 8) | (widx << 16);
}

// Optional BatchNorm-backward partials of a dgrad OUTPUT (X != nullptr): when the convolution's input
// was relu(bn(X)) (a BasicBlock's conv2 input a1 = relu(bn1(y1))), the dgrad output is bn1's dA, and
// its backward reduction -- per channel (sum d, sum d * xhat), d = dA * (X*sc + sh > 0), xhat =
// (X - mu) * rs -- is summed here, in the store loop, from the rounded bf16 output and one 16-B read
// of X per chunk, into part[mtile][2][NC] (the k_bn_bwd_reduce<2> format): no separate pass re-reading
// dA.  Same per-element math as k_bn_bwd_reduce<2>; per-tile sums in a fixed order (deterministic).
struct BnbArgs {
  const bf16_t* X;
  const float *sc, *sh, *mu, *rs;
  float* part;
};

// Store-loop side: this thread's 8 channels (chunk n8 = first channel) of one output row.
struct BnbAcc {
  float s[8], q[8], sc[8], sh[8], mu[8], rs[8];
  // per-channel constants: issue early (an epilogue-time load stalls the block one memory latency)
  __device__ __forceinline__ void init(const BnbArgs& z, int n8) {
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      sc[e] = z.sc[n8 + e];
      sh[e] = z.sh[n8 + e];
      mu[e] = z.mu[n8 + e];
      rs[e] = z.rs[n8 + e];
    }
    reset();
  }
  __device__ __forceinline__ void reset() {
#pragma unroll
    for (int e = 0; e < 8; ++e) s[e] = q[e] = 0.f;
  }
  __device__ __forceinline__ void add(uint4 out, uint4 xin) {
    float g[8], x[8];
    unpack8(out, g);
    unpack8(xin, x);
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float d = x[e] * sc[e] + sh[e] > 0.f ? g[e] : 0.f;
      s[e] += d;
      q[e] += d * (x[e] - mu[e]) * rs[e];
    }
  }
  // Fold the lanes of each wave that share this chunk (lane % CPR), then the waves through LDS
  // red[NW][2][BN]; threads < 2 BN write row `row` of part.  Call from every thread of the block.
  template <int CPR, int NW, int BN>
  __device__ __forceinline__ void flush(float* red, const BnbArgs& z, size_t row, int NC, int n0) {
    const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);   // w wave-uniform
#pragma unroll
    for (int off = CPR; off < 64; off <<= 1)
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        s[e] += __shfl_xor(s[e], off, 64);
        q[e] += __shfl_xor(q[e], off, 64);
      }
    if (l < CPR) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        red[(w * 2 + 0) * BN + l * 8 + e] = s[e];
        red[(w * 2 + 1) * BN + l * 8 + e] = q[e];
      }
    }
    __syncthreads();
    if (t < 2 * BN) {
      const int which = t / BN, n = t % BN;
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < NW; ++k) a += red[(k * 2 + which) * BN + n];
      z.part[(row * 2 + which) * NC + n0 + n] = a;
    }
  }
};

struct IgemmArgs {
  const bf16_t* A;      // gather source NHWC [Bn][IH][IW][CA]
  const bf16_t* W;      // [NC][T][CA]
  bf16_t* Y;            // NHWC [Bn][OH][OW][NC]
  const bf16_t* R;      // optional, same layout as Y: Y = bf16(acc) + R (residual-gradient accumulate)
  // optional second K source (dgrad of a ResNet block's 1x1 / stride-2 downsample, folded into the
  // block's conv1 dgrad): A2 is shaped like A and read at tap delta (0, 0) (the output pixel's own
  // position), W2 = [NC][1][CA]; phases with ntap2 = 1 append CA / 64 stages over it
  const bf16_t* A2;
  const bf16_t* W2;
  uint32_t a2_bytes, w2_bytes;
  float* stats;         // optional [mtiles][2][NC] (single-phase launches)
  BnbArgs bnb;          // optional BN-backward partials of the output (single-phase launches)
  uint32_t a_bytes, w_bytes;
  int Bn, IH, IW, CA;
  int OH, OW, NC, T;
  int sA, sO;           // source pixel = q * sA + d ; output pixel = q * sO + phase offset
  int nphase, mtiles, ntiles;
  Phase phase[4];
};

constexpr int kThreads = 256;

// Pipeline: NST LDS stage buffers filled by LDS-DMA, NST-1 stages in flight ahead of the MFMAs.
// Per stage: wait for this wave's DMA of the stage (counted vmcnt, never a blanket drain while a
// younger stage is in flight), raw s_barrier (every wave's DMA for the stage has landed, and every
// wave is done reading the buffer about to be refilled), issue the stage NST-1 ahead, compute.
template <int BM, int BN, int NST>
__global__ __launch_bounds__(kThreads, NST == 2 ? 2 : 1) void k_igemm(IgemmArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  static_assert(WM * 64 == BM, "wave grid must tile BM x BN with 64x64 wave tiles");
  constexpr int AI = BM / 32, BI = BN / 32;         // glds wave-instructions per wave per stage
  constexpr int LPS = AI + BI;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, STAGE = ABYTES + BBYTES;
  constexpr int RS = BN * 2 + 16;                    // epilogue LDS row stride (bytes)
  constexpr int EPI = BM * RS + 2 * WM * BN * 4;
  constexpr int EPIR = EPI + 4 * 2 * BN * 4;         // + the BN-backward fold red[4][2][BN]
  constexpr int SMEM = NST * STAGE > EPIR ? NST * STAGE : EPIR;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);   // w wave-uniform
  const int nwg = gridDim.x;
  const int id = xcd_remap(blockIdx.x, nwg);
  // phases interleaved in the block id: each XCD (a contiguous id range, xcd_remap) gets an equal share
  // of every phase.  Phase-major ids gave the 4-tap phase of a stride-2 dgrad (1, 2, 2, 4 taps) to
  // XCDs 6-7 alone, which then ran ~1.6x the balanced time.
  const int phz = id % a.nphase, rem = id / a.nphase;
  const int mt = rem / a.ntiles, nt = rem % a.ntiles;
  const Phase& P = a.phase[phz];
  const int Mq = a.Bn * P.Hq * P.Wq;
  const int m0 = mt * BM, n0 = nt * BN;
  if (m0 >= Mq) return;                              // whole block (phase grids differ in size)
  const int CPT = a.CA >> 6;                         // 64-channel stages per tap
  const int KT1 = P.ntap * CPT;
  const int KT = KT1 + P.ntap2 * CPT;
  const int ldw = a.T * a.CA;

  // ---- per-thread gather rows: instruction i fills 8-row group 4i + w, this lane row glds_row ----
  const int lrow = glds_row(l), ch = glds_chunk(l, w & 1);
  // Per row: element offset of its pixel (tap delta 0) + this lane's channel chunk, and a bit per tap
  // telling whether that tap lies inside the image.  Per stage the tap's offset delta is
  // wave-uniform (scalar), so a row's load costs one add, a bit test and a select (VALU per MFMA
  // was the limiter of the first version: 22 vector instructions per MFMA at BM = 256).
  int aoff[AI];
  uint32_t vmask[AI];
  int taps[9];
#pragma unroll
  for (int tt = 0; tt < 9; ++tt) taps[tt] = P.tap[tt];     // wave-uniform, loaded once
#pragma unroll
  for (int u = 0; u < AI; ++u) {
    const int m = m0 + 8 * (4 * u + w) + lrow;
    aoff[u] = 0;
    vmask[u] = 0;
    if (m < Mq) {
      const int b = fdiv(m, P.Hq * P.Wq, P.inv_hw), r2 = m - b * (P.Hq * P.Wq);
      const int hq = fdiv(r2, P.Wq, P.inv_w), wq = r2 - hq * P.Wq;
      const int hb = hq * a.sA, wb = wq * a.sA;
      aoff[u] = ((b * a.IH + hb) * a.IW + wb) * a.CA + ch * 8;
      uint32_t mk = 0;
#pragma unroll
      for (int tt = 0; tt < 9; ++tt) {
        const int tp = taps[tt];
        const int ih = hb + (int)(signed char)(tp & 0xff), iw = wb + (int)(signed char)((tp >> 8) & 0xff);
        mk |= (tt < P.ntap && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW) ? (1u << tt) : 0u;
      }
      // bit 9: the pixel's own position (the second source's only tap)
      mk |= ((unsigned)hb < (unsigned)a.IH && (unsigned)wb < (unsigned)a.IW) ? (1u << 9) : 0u;
      vmask[u] = mk;
    }
  }
  const rsrc_t ar = make_rsrc(a.A, a.a_bytes), wr = make_rsrc(a.W, a.w_bytes);
  uint32_t wrow[BI];
#pragma unroll
  for (int v = 0; v < BI; ++v) wrow[v] = ((n0 + 8 * (4 * v + w) + lrow) * ldw + ch * 8) * 2;
  const rsrc_t ar2 = make_rsrc(a.A2, a.a2_bytes), wr2 = make_rsrc(a.W2, a.w2_bytes);

  auto issue = [&](int kt, int buf) {
    if (kt >= KT1) {                                   // second source: own position, W2 rows of CA
      const int c0 = (kt - KT1) * 64;
      const char* Ai = smem + buf * STAGE;
      const char* Bi = Ai + ABYTES;
#pragma unroll
      for (int u = 0; u < AI; ++u) {
        const bool ok = (vmask[u] >> 9) & 1u;
        glds16(ar2, Ai + (4 * u + w) * 1024, ok ? (uint32_t)(aoff[u] + c0) * 2u : kOOB);
      }
#pragma unroll
      for (int v = 0; v < BI; ++v)
        glds16(wr2, Bi + (4 * v + w) * 1024, (uint32_t)(((n0 + 8 * (4 * v + w) + lrow) * a.CA + ch * 8 + c0) * 2));
      return;
    }
    const int tap = kt / CPT, c0 = (kt - tap * CPT) * 64;
    const int tp = P.tap[tap];
    const int dh = (int)(signed char)(tp & 0xff), dw = (int)(signed char)((tp >> 8) & 0xff), wi = tp >> 16;
    const int td = (dh * a.IW + dw) * a.CA + c0;     // wave-uniform
    const char* Ai = smem + buf * STAGE;
    const char* Bi = Ai + ABYTES;
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const bool ok = (vmask[u] >> tap) & 1u;
      glds16(ar, Ai + (4 * u + w) * 1024, ok ? (uint32_t)(aoff[u] + td) * 2u : kOOB);
    }
#pragma unroll
    for (int v = 0; v < BI; ++v) glds16(wr, Bi + (4 * v + w) * 1024, wrow[v] + (uint32_t)(wi * a.CA + c0) * 2u);
  };

  const int wm = w / WN, wn = w % WN, lr = l & 31, lh = l >> 5;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0.f};

  if (KT > 0) {
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
      if (s < KT) issue(s, s);
    int buf = 0;
    for (int kt = 0; kt < KT; ++kt) {
      if constexpr (NST >= 3) {
        if (kt + 1 < KT) wait_vm<LPS>();
        else wait_vm<0>();
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      if (kt + NST - 1 < KT) {
        int nb = buf + NST - 1;
        nb = nb >= NST ? nb - NST : nb;
        issue(kt + NST - 1, nb);
      }
      const char* Ai = smem + buf * STAGE;
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
      buf = buf + 1 == NST ? 0 : buf + 1;
    }
    __syncthreads();                                   // every wave is done with the stage buffers
  }

  // ---- epilogue: bf16 tile through LDS, coalesced NHWC rows; optional BN partial stats ----
  const bool bnb = a.bnb.X != nullptr;
  BnbAcc za;
  if (bnb) za.init(a.bnb, n0 + (t % (BN / 8)) * 8);  // a thread's chunk is fixed (kThreads % CPR == 0)
  char* ot = smem;
  float* sst = reinterpret_cast<float*>(smem + BM * RS);   // [WM][2][BN]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = wn * 64 + j * 32 + lr;
      bf16_t hv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = wm * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
        hv[q] = f2bf(acc[i][j][q]);
        *reinterpret_cast<bf16_t*>(ot + m * RS + n * 2) = hv[q];
      }
      if (a.stats) {   // (rows past Mq are zero: their A rows were zero-filled)
        float s1 = 0.f, s2 = 0.f;
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const float fv = bf2f(hv[q]);
          s1 += fv;
          s2 += fv * fv;
        }
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
  constexpr int EU = BM * CPR / kThreads;
  // the epilogue's second input (residual gradient R, or the BN input X; never both) is prefetched
  // for every chunk before the first store: loads issued inside the store loop were serialised behind
  // the stores (possible aliasing), one memory latency per chunk
  const bf16_t* pf = bnb ? a.bnb.X : a.R;
  size_t oo[EU];
  uint4 pre[EU];
#pragma unroll
  for (int u = 0; u < EU; ++u) {
    const int c = t + kThreads * u, row = c / CPR, cc = c % CPR;
    const int m = min(m0 + row, Mq - 1);               // rows past Mq are never stored
    const int b = fdiv(m, P.Hq * P.Wq, P.inv_hw), r2 = m - b * (P.Hq * P.Wq);
    const int hq = fdiv(r2, P.Wq, P.inv_w);
    const int oh = hq * a.sO + P.ph, ow = (r2 - hq * P.Wq) * a.sO + P.pw;
    oo[u] = (((size_t)b * a.OH + oh) * a.OW + ow) * a.NC + n0 + cc * 8;
    if (pf) pre[u] = *reinterpret_cast<const uint4*>(pf + oo[u]);
  }
#pragma unroll
  for (int u = 0; u < EU; ++u) {
    const int c = t + kThreads * u, row = c / CPR, cc = c % CPR;
    if (m0 + row < Mq) {
      uint4 v = *reinterpret_cast<const uint4*>(ot + row * RS + cc * 16);
      const size_t o = oo[u];
      if (a.R) {                                       // the other consumer's gradient, added once
        float f[8], r[8];
        unpack8(v, f);
        unpack8(pre[u], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += r[e];
        v = pack8(f);
      }
      *reinterpret_cast<uint4*>(a.Y + o) = v;
      if (bnb) za.add(v, pre[u]);
    }
  }
  if (bnb) za.flush<CPR, 4, BN>(reinterpret_cast<float*>(smem + EPI), a.bnb, (size_t)mt, a.NC, n0);
  if (a.stats && t < 2 * BN) {
    const int which = t / BN, n = t % BN;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WM; ++k) s += sst[(k * 2 + which) * BN + n];
    a.stats[((size_t)mt * 2 + which) * a.NC + n0 + n] = s;
  }
}

// Wt[c][t][n] = W[n][t][c]  (64x64 tiles through LDS; grid (C/64, N/64, T))
__device__ __forceinline__ void wtrans_tile(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wt, int N, int T,
                                            int C, int c0, int n0, int tap) {
  __shared__ bf16_t sh[64][66];
  const int t = threadIdx.x;
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

__global__ __launch_bounds__(256) void k_wtrans(const bf16_t* __restrict__ W, bf16_t* __restrict__ Wt, int N,
                                                int T, int C) {
  wtrans_tile(W, Wt, N, T, C, blockIdx.x * 64, blockIdx.y * 64, blockIdx.z);
}

// All dgrad weight transposes of a network in ONE launch (one per step instead of one per conv
// backward): block b finds its convolution in the descriptor table by a scan of the tile offsets.
struct WtDesc {
  const bf16_t* w;
  bf16_t* wt;
  int N, T, C, tile0;
};
// ctr (nullable): ncnt int64 counters bumped by block 0 -- the model's BatchNorm num_batches_tracked,
// advanced by this once-per-training-forward launch instead of an ATen add kernel
__global__ __launch_bounds__(256) void k_wtrans_batch(const WtDesc* __restrict__ d, int nconv,
                                                      long long* __restrict__ ctr, int ncnt) {
  const int b = blockIdx.x;
  if (ctr && b == 0 && (int)threadIdx.x < ncnt) ctr[threadIdx.x] += 1;
  int i = 0;
  while (i + 1 < nconv && d[i + 1].tile0 <= b) ++i;
  const WtDesc& q = d[i];
  const int lt = b - q.tile0, cb = q.C >> 6, nb = q.N >> 6;
  const int cx = lt % cb, ny = (lt / cb) % nb, tap = lt / (cb * nb);
  wtrans_tile(q.w, q.wt, q.N, q.T, q.C, cx * 64, ny * 64, tap);
}

// ============================================================================ wgrad
struct WgradArgs {
  const bf16_t* dY;     // [P][N]
  const bf16_t* X;      // [Bn][IH][IW][C]
  float* part;          // [splits][N][T*C]
  uint32_t dy_bytes, x_bytes;
  int Bn, IH, IW, C, OH, OW, N, S, stride, pad, T;
  int P, stages_per_split, mtiles, ntiles;
  float inv_hw, inv_w;
  int incr;             // unused (the walk is the kernel's INC template flag)
};

template <int BM, int BN, int NST, bool INC>
__global__ __launch_bounds__(kThreads, NST == 2 ? 2 : 1) void k_wgrad(WgradArgs a) {
  constexpr int WN = (BN / 64 >= 4) ? 4 : BN / 64;   // waves along the (tap, c) columns
  constexpr int WM = 4 / WN;
  constexpr int TM = BM / WM / 32, TN = BN / WN / 32;
  static_assert(TM >= 1 && TN >= 1 && WM * WN == 4, "wgrad tiling");
  constexpr int ABYTES = (BM / 64) * 8192, BBYTES = (BN / 64) * 8192, STAGE = ABYTES + BBYTES;
  constexpr int AI = BM / 32, BI = BN / 32;          // glds wave-instructions per wave per stage
  constexpr int LPS = AI + BI;
  __shared__ __attribute__((aligned(16))) char smem[NST * STAGE];

  // w through readfirstlane: the compiler then knows it is wave-uniform, so every LDS-DMA destination
  // (m0) and row-group index derived from it is scalar arithmetic instead of VALU + v_readfirstlane
  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = a.mtiles * a.ntiles;
  const int split = id / ntile, rem = id % ntile;
  const int mt = rem / a.ntiles, nt = rem % a.ntiles;
  const int n0 = mt * BM, k0 = nt * BN;              // output rows (Cout) / columns (tap, c)
  const int TC = a.T * a.C;
  const int pbeg = split * a.stages_per_split * 64;
  const int pend = min(a.P, pbeg + a.stages_per_split * 64);
  const int KT = (pend - pbeg + 63) / 64;

  // instruction u fills 8-row group (4u + w) % 8 of 64-column image (4u + w) / 8
  const int lrow = glds_row(l), ch = glds_chunk(l, w & 1);
  int xr_[BI], xs_[BI], xc_[BI];
#pragma unroll
  for (int v = 0; v < BI; ++v) {
    const int col = k0 + ((4 * v + w) >> 3) * 64 + ch * 8;
    const bool ok = col < TC;
    const int cc = min(col, TC - 1);
    const int tap = cc / a.C;
    xc_[v] = cc - tap * a.C;
    xr_[v] = ok ? tap / a.S - a.pad : -(1 << 20);    // a column past T*C reads zeros
    xs_[v] = tap % a.S - a.pad;
  }
  const rsrc_t dyr = make_rsrc(a.dY, a.dy_bytes), xr = make_rsrc(a.X, a.x_bytes);
  // B rows (INC, 64 / OW + 1 < 2 OH): instructions v and v + 2 load the same 8 pixel rows ((4 v + w) & 7)
  // for the two 64-column images, so NR = 2 row walks serve all BI instructions.  A walk keeps
  // (pb, poh, pow_) = (element offset of x[b][oh s][ow s][0], oh s, ow s) of its lane's row, decomposed
  // once and advanced by 64 pixels per issued stage with uniform deltas -- wd0, + wdw on a column wrap,
  // + wdh per row wrap (at most one carry into oh, two into b) -- and an instruction's address is the
  // walk's offset + its per-lane tap offset toff[v] = (dr IW + ds) C + c.  No divisions and no
  // multiplies in the loop (v_mul_lo_u32 is quarter rate): the former walk per instruction with a
  // multiply-formed address cost ~230 VALU per 16 MFMAs (profiles/r5_models/wgrad_shared_walk/).
  const int dq64 = 64 / a.OW, dr64 = 64 - dq64 * a.OW;
  constexpr int NR = BI >= 2 ? 2 : 1;
  int pb[NR], poh[NR], pow_[NR];
  int toff[BI];
#pragma unroll
  for (int v = 0; v < BI; ++v) toff[v] = xr_[v] > -(1 << 19) ? (xr_[v] * a.IW + xs_[v]) * a.C + xc_[v] : 0;
  const int wow = a.OW * a.stride, woh = a.OH * a.stride, wdr = dr64 * a.stride, wdq = dq64 * a.stride;
  const int wd0 = (dq64 * a.stride * a.IW + dr64 * a.stride) * a.C;
  const int wdw = (a.stride * a.IW - wow) * a.C, wdh = (a.IH - woh) * a.IW * a.C;
  if constexpr (INC) {
#pragma unroll
    for (int r = 0; r < NR; ++r) {
      const int p = pbeg + 8 * ((4 * r + w) & 7) + lrow;
      const int b = p / (a.OH * a.OW), r2 = p - b * (a.OH * a.OW);
      const int oh = r2 / a.OW, ow = r2 - oh * a.OW;
      poh[r] = oh * a.stride;
      pow_[r] = ow * a.stride;
      pb[r] = ((b * a.IH + poh[r]) * a.IW + pow_[r]) * a.C;
    }
  }
  auto issue = [&](int kt, int buf) {
    const int p0 = pbeg + kt * 64;
    const char* Ai = smem + buf * STAGE;
    const char* Bi = Ai + ABYTES;
#pragma unroll
    for (int u = 0; u < AI; ++u) {
      const int q = 4 * u + w, p = p0 + 8 * (q & 7) + lrow;
      const uint32_t off = (uint32_t)(p * a.N + n0 + (q >> 3) * 64 + ch * 8) * 2u;
      glds16(dyr, Ai + q * 1024, p < pend ? off : kOOB);
    }
    if constexpr (INC) {
#pragma unroll
      for (int v = 0; v < BI; ++v) {
        const int q = 4 * v + w, r = v % NR;
        const bool pin = p0 + 8 * ((4 * r + w) & 7) + lrow < pend;
        const bool ok = pin & ((unsigned)(poh[r] + xr_[v]) < (unsigned)a.IH) &   // & : no short-circuit
                        ((unsigned)(pow_[r] + xs_[v]) < (unsigned)a.IW);           // exec-mask branches
        glds16(xr, Bi + q * 1024, ok ? (uint32_t)(pb[r] + toff[v]) * 2u : kOOB);
      }
      // advance by 64 pixels: no multiplies (v_mul_lo_u32 is quarter rate), the deltas are uniform
#pragma unroll
      for (int r = 0; r < NR; ++r) {
        int ows = pow_[r] + wdr, ohs = poh[r] + wdq, rb = pb[r] + wd0;
        if (ows >= wow) { ows -= wow; ohs += a.stride; rb += wdw; }
        if (ohs >= woh) { ohs -= woh; rb += wdh; }
        if (ohs >= woh) { ohs -= woh; rb += wdh; }
        pow_[r] = ows;
        poh[r] = ohs;
        pb[r] = rb;
      }
      return;
    }
#pragma unroll
    for (int v = 0; v < BI; ++v) {
      const int q = 4 * v + w, p = p0 + 8 * (q & 7) + lrow;
      const int pp = min(p, a.P - 1);  // (walk precondition 64 / OW + 1 < 2 OH fails: tiny images)
      const int b = fdiv(pp, a.OH * a.OW, a.inv_hw);
      const int r2 = pp - b * (a.OH * a.OW);
      const int oh = fdiv(r2, a.OW, a.inv_w);
      const int ow = r2 - oh * a.OW;
      const int ih = oh * a.stride + xr_[v], iw = ow * a.stride + xs_[v];
      const bool ok = p < pend && (unsigned)ih < (unsigned)a.IH && (unsigned)iw < (unsigned)a.IW;
      const uint32_t off = (uint32_t)(((b * a.IH + ih) * a.IW + iw) * a.C + xc_[v]) * 2u;
      glds16(xr, Bi + q * 1024, ok ? off : kOOB);
    }
  };

  const int wm = w / WN, wn = w % WN, lr = l & 31;
  // per-wave transposed-read bases (the fragment column offsets separate: BM/WM, BN/WN are 32 or 64)
  static_assert((BM / WM) % 64 == 0 || TM == 1, "A column blocks");
  static_assert((BN / WN) % 64 == 0 || TN == 1, "B column blocks");
  const uint32_t lds_base = (uint32_t)(uintptr_t)(lds_char*)smem;
  const uint2 a_lane = add2(tr_lane_off(), colblk_off(wm * (BM / WM) / 32));
  const uint2 b_lane = add2(tr_lane_off(), colblk_off(wn * (BN / WN) / 32));
  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{0.f};

  if (KT > 0) {
#pragma unroll
    for (int s = 0; s < NST - 1; ++s)
      if (s < KT) issue(s, s);
    int buf = 0;
    for (int kt = 0; kt < KT; ++kt) {
      if constexpr (NST >= 3) {
        if (kt + 1 < KT) wait_vm<LPS>();
        else wait_vm<0>();
      } else {
        wait_vm<0>();
      }
      __builtin_amdgcn_s_barrier();
      if (kt + NST - 1 < KT) {
        int nb = buf + NST - 1;
        nb = nb >= NST ? nb - NST : nb;
        issue(kt + NST - 1, nb);
      }
      // fragments of k-step s+1 are read while the MFMAs of k-step s run (two named register sets)
      const uint32_t sb = lds_base + buf * STAGE;
      const uint2 ab = add2(a_lane, sb), bb = add2(b_lane, sb + ABYTES);
      bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
      auto mm = [&](const bf16x8* fa, const bf16x8* fb) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
      };
      wg_frags<0, TM, TN>(ab, bb, fa0, fb0);
      lgkm_fence();
      wg_frags<1, TM, TN>(ab, bb, fa1, fb1);
      mm(fa0, fb0);
      lgkm_fence();
      wg_frags<2, TM, TN>(ab, bb, fa0, fb0);
      mm(fa1, fb1);
      lgkm_fence();
      wg_frags<3, TM, TN>(ab, bb, fa1, fb1);
      mm(fa0, fb0);
      lgkm_fence();
      mm(fa1, fb1);
      buf = buf + 1 == NST ? 0 : buf + 1;
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

// ============================================================================ halo-tiled 3x3 / stride 1
// The implicit GEMM above re-fetches its A operand through L2 once per tap (9x for a 3x3 conv): at
// C = 64 (layer1) a stage is 40 KB of DMA for 2 MFLOP, and the kernel runs at the L2 -> LDS rate.
// k_hconv stages, per 64-channel chunk, the HALO of a block of TH full output rows once --
// (TH + 2) x (W + 2) input pixels, out-of-image pixels zero-filled by the bounded buffer load -- and
// reads all nine taps' A fragments from it (a tap is a constant shift of the halo pixel index), so
// only the weights stream per tap (double-buffered).  Block = TH rows x W columns of output pixels
// (<= BM, rounded up to MFMA tiles), BN output channels; 4 waves of 64 x 64 as in k_igemm, and the
// same epilogue (bf16 tile through LDS, BN statistics partials, residual add).  Used for stride-1
// 3x3 / pad-1 fprop and dgrad (the dgrad of a stride-1 conv is the flipped-tap conv of dy with Wt).
struct HconvArgs {
  const bf16_t* A;      // NHWC [Bn][H][W][CA]
  const bf16_t* Wg;     // [NC][9][CA]
  bf16_t* Y;            // NHWC [Bn][H][W][NC]
  const bf16_t* R;      // optional, like Y: Y = bf16(acc) + R
  float* stats;         // optional [Bn * rtiles][2][NC]
  BnbArgs bnb;          // optional BN-backward partials of the output, [Bn * rtiles][2][NC]
  uint32_t a_bytes, w_bytes;
  int Bn, H, W, CA, NC;
  int TH, rtiles, ntiles;
  int tap[9];           // pack_tap(dh, dw, widx)
};

template <int BM> constexpr int hconv_groups() { return BM == 256 ? 50 : 33; }   // 8-pixel halo groups

// Halo image layout: pixel row r at r * 128 B, 16-byte channel chunk c in slot c ^ hsw((r >> 1) & 7) with
// hsw(v) = (v0 << 2) | v1 << 1 | v2 (bit-reversed v).  A tap shifts the rows a wave reads by an
// arbitrary amount, so the image must be conflict-free for unaligned rows, for two access shapes:
//  * ds_read_b128 row fragments (k_hconv A): 16 consecutive rows, one chunk -> per bank half (r & 1)
//    8 consecutive v, hsw a bijection -> 8 distinct slots;
//  * ds_read_b64_tr_b16 (k_hwgrad64): 4 consecutive rows x a 4-chunk half (c..c+3, c = 0 or 4) -> the
//    two rows sharing a bank half have consecutive v, whose hsw differ in bit 2 (= v0), so their 4-slot
//    sets land in opposite halves of the row.
// (The first version, c ^ v, mapped a chunk pair onto itself for v, v+1: 1.8 conflict cycles per LDS
// instruction in the transposed reads.)  LDS-DMA fills a 1 KB group lane-linearly: lane l -> row
// l >> 3 of the group, slot l & 7.
__device__ __forceinline__ int hsw(int v) { return ((v & 1) << 2) | (v & 2) | ((v >> 2) & 1); }
__device__ __forceinline__ bf16x8 halo_frag(const char* halo, int row, int chunk) {
  return *reinterpret_cast<const bf16x8*>(halo + row * 128 + 16 * (chunk ^ hsw((row >> 1) & 7)));
}
// channel chunk that lane l loads for halo group g (parity gpar = g & 1; groups are 8 rows)
__device__ __forceinline__ int halo_dma_chunk(int l, int gpar) { return (l & 7) ^ hsw((4 * gpar + (l >> 4)) & 7); }

template <int BM, int BN, int V>
__global__ __launch_bounds__(kThreads, 2) void k_hconv(HconvArgs a) {
  constexpr int WN = BN / 64, WM = 4 / WN;
  static_assert(WM * 64 == BM, "wave grid must tile BM x BN with 64x64 wave tiles");
  constexpr int HG = hconv_groups<BM>(), HU = (HG + 3) / 4;   // halo groups, glds per wave
  constexpr int HBYTES = HG * 1024;
  constexpr int BI = BN / 32, BBYTES = BN * 128;
  constexpr int RS = BN * 2 + 16;
  constexpr int EPIB = BM * RS + 2 * WM * BN * 4;
  constexpr int EPIR = EPIB + 4 * 2 * BN * 4;        // + the BN-backward fold red[4][2][BN]
  constexpr int SMEM = HBYTES + 2 * BBYTES > EPIR ? HBYTES + 2 * BBYTES : EPIR;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];
  char* halo = smem;
  char* bimg = smem + HBYTES;

  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);   // w wave-uniform
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int nt = id % a.ntiles, mt = id / a.ntiles;
  const int b = mt / a.rtiles, rt = mt - b * a.rtiles;
  const int oh0 = rt * a.TH, rows = min(a.TH, a.H - oh0), npx = rows * a.W;
  const int n0 = nt * BN, HW2 = a.W + 2;
  const int CPT = a.CA >> 6, ldw = 9 * a.CA;

  // ---- halo DMA sources: group g = w + 4u, lane row glds_row, chunk glds_chunk (group parity = w & 1) ----
  const int lrow = glds_row(l), ch = glds_chunk(l, w & 1);
  const int hrow = l >> 3, hch = halo_dma_chunk(l, w & 1);   // halo groups w + 4u share parity w & 1
  uint32_t hoff[HU];
#pragma unroll
  for (int u = 0; u < HU; ++u) {
    const int hr = 8 * (w + 4 * u) + hrow;
    const int hy = hr / HW2, hx = hr - hy * HW2;
    const int ih = oh0 - 1 + hy, iw = hx - 1;
    const bool ok = hy < a.TH + 2 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
    hoff[u] = ok ? (uint32_t)((((b * a.H + ih) * a.W + iw) * a.CA + hch * 8) * 2) : kOOB;
  }
  uint32_t wrow[BI];
#pragma unroll
  for (int v = 0; v < BI; ++v) wrow[v] = (uint32_t)(((n0 + 8 * (4 * v + w) + lrow) * ldw + ch * 8) * 2);
  const rsrc_t ar = make_rsrc(a.A, a.a_bytes), wr = make_rsrc(a.Wg, a.w_bytes);

  // ---- this lane's MFMA A rows: pixel p of tile i -> halo index of its tap-(0,0) input ----
  const int wm = w / WN, wn = w % WN, lr = l & 31, lh = l >> 5;
  int hbase[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    int p = wm * 64 + i * 32 + lr;
    p = p < npx ? p : 0;                               // masked in the epilogue
    const int py = p / a.W, px = p - py * a.W;
    hbase[i] = (py + 1) * HW2 + px + 1;
  }

  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0.f};

  auto issue_b = [&](int tap, int c0, int buf) {
    const int wi = a.tap[tap] >> 16;
#pragma unroll
    for (int v = 0; v < BI; ++v)
      glds16(wr, bimg + buf * BBYTES + (4 * v + w) * 1024, wrow[v] + (uint32_t)((wi * a.CA + c0) * 2));
  };

  // the epilogue's second input (residual gradient or BN input, never both): loaded with the last
  // channel chunk's halo, so it lands under that chunk's MFMAs instead of stalling the epilogue
  constexpr int CPR = BN / 8, EU = BM * CPR / kThreads;
  const size_t obase = ((size_t)b * a.H + oh0) * a.W;     // first output pixel of the block
  const bool bnb = a.bnb.X != nullptr;
  const bf16_t* pf = bnb ? a.bnb.X : a.R;
  uint4 pre[EU];
  BnbAcc za;
  for (int cc = 0; cc < CPT; ++cc) {
    const int c0 = cc * 64;
    if (cc > 0) __syncthreads();                       // every wave is done with the previous chunk
#pragma unroll
    for (int u = 0; u < HU; ++u)
      if (w + 4 * u < HG) glds16(ar, halo + (w + 4 * u) * 1024, hoff[u] == kOOB ? kOOB : hoff[u] + c0 * 2);
    if (pf && cc == CPT - 1) {
#pragma unroll
      for (int u = 0; u < EU; ++u) {
        const int c = t + kThreads * u, row = min(c / CPR, npx - 1);
        pre[u] = *reinterpret_cast<const uint4*>(pf + (obase + row) * a.NC + n0 + (c % CPR) * 8);
      }
    }
    issue_b(0, c0, 0);
    if constexpr (V == 0) {
      for (int tp = 0; tp < 9; ++tp) {
        wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (tp + 1 < 9) issue_b(tp + 1, c0, (tp + 1) & 1);
        const int pk = a.tap[tp];
        const int td = (int)(signed char)(pk & 0xff) * HW2 + (int)(signed char)((pk >> 8) & 0xff);
        const char* Bi = bimg + (tp & 1) * BBYTES;
        int hp[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) hp[i] = hbase[i] + td;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          bf16x8 fa[2], fb[2];
#pragma unroll
          for (int i = 0; i < 2; ++i) fa[i] = halo_frag(halo, hp[i], 2 * s4 + lh);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[j] = row_frag(Bi, wn * 64 + j * 32 + lr, 2 * s4 + lh);
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
        }
      }
    } else {
      // V = 1 (default): the A-fragment row bases pass through an opaque register move at every tap,
      // so the compiler cannot hoist all 9 taps x 8 fragment addresses out of the channel loop (V = 0:
      // 72 VGPRs at the 256-register cap, leaving 12 for fragments and an lgkmcnt wait in front of
      // nearly every MFMA; V = 1: 217 VGPRs, 72 instead of 108 waits per chunk, ~33 more VALU per tap).
      // l2 / l3 convs 3-5 % faster, ResNet-18 step +0.7 % (profiles/r5_models/hconv_tap_addresses/).
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        if (tp + 1 < 9) issue_b(tp + 1, c0, (tp + 1) & 1);
        const int pk = a.tap[tp];
        const int td = (int)(signed char)(pk & 0xff) * HW2 + (int)(signed char)((pk >> 8) & 0xff);
        const char* Bi = bimg + (tp & 1) * BBYTES;
        // halo_frag(halo, row, 2 s4 + lh) = halo + (row * 128 + 16 (lh ^ key)) ^ 32 s4: one XOR per
        // fragment address once the s4 = 0 address is formed
        int ha[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          int row = hbase[i];
          asm volatile("" : "+v"(row));
          row += td;
          ha[i] = row * 128 + 16 * (lh ^ hsw((row >> 1) & 7));
        }
        bf16x8 fa[4][2], fb[4][2];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
#pragma unroll
          for (int i = 0; i < 2; ++i) fa[s4][i] = *reinterpret_cast<const bf16x8*>(halo + (ha[i] ^ (32 * s4)));
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[s4][j] = row_frag(Bi, wn * 64 + j * 32 + lr, 2 * s4 + lh);
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(fa[s4][i], fb[s4][j], acc[i][j]);
      }
    }
  }
  __syncthreads();                                     // every wave is done with the halo / weights

  // ---- epilogue (as k_igemm): bf16 tile through LDS, masked BN partials, coalesced NHWC rows ----
  if (bnb) za.init(a.bnb, n0 + (t % CPR) * 8);        // lands under the tile conversion below
  char* ot = smem;
  float* sst = reinterpret_cast<float*>(smem + BM * RS);   // [WM][2][BN]
  // statistics only when requested (the dgrad launches have none), the row mask only where this
  // 32-row fragment runs past npx: wave-uniform branches (as k_hconv64)
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int n = wn * 64 + j * 32 + lr;
      bf16_t hv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int m = wm * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
        hv[q] = f2bf(acc[i][j][q]);
        *reinterpret_cast<bf16_t*>(ot + m * RS + n * 2) = hv[q];
      }
      if (a.stats) {
        float s1 = 0.f, s2 = 0.f;
        if (wm * 64 + i * 32 + 32 <= npx) {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const float fv = bf2f(hv[q]);
            s1 += fv;
            s2 += fv * fv;
          }
        } else {
#pragma unroll
          for (int q = 0; q < 16; ++q) {
            const int m = wm * 64 + i * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
            const float fv = m < npx ? bf2f(hv[q]) : 0.f;
            s1 += fv;
            s2 += fv * fv;
          }
        }
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
#pragma unroll
  for (int u = 0; u < EU; ++u) {
    const int c = t + kThreads * u, row = c / CPR, cc = c % CPR;
    if (row < npx) {
      uint4 v = *reinterpret_cast<const uint4*>(ot + row * RS + cc * 16);
      const size_t o = (obase + row) * a.NC + n0 + cc * 8;
      if (a.R) {
        float f[8], r[8];
        unpack8(v, f);
        unpack8(pre[u], r);
#pragma unroll
        for (int e = 0; e < 8; ++e) f[e] += r[e];
        v = pack8(f);
      }
      *reinterpret_cast<uint4*>(a.Y + o) = v;
      if (bnb) za.add(v, pre[u]);
    }
  }
  if (bnb) za.flush<CPR, 4, BN>(reinterpret_cast<float*>(smem + EPIB), a.bnb, (size_t)mt, a.NC, n0);
  if (a.stats && t < 2 * BN) {
    const int which = t / BN, n = t % BN;
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < WM; ++k) s += sst[(k * 2 + which) * BN + n];
    a.stats[((size_t)mt * 2 + which) * a.NC + n0 + n] = s;
  }
}

// Persistent variant for C = NC = 64 (ResNet-18 layer1, fprop and dgrad): the whole 3x3 weight
// (9 taps x [64][64] bf16 = 72 KB) is staged ONCE per block and stays in LDS; the block then walks
// its row tiles (tile = blockIdx.x + k * gridDim.x) with the halo double-buffered, so the next tile's
// halo DMA runs under this tile's 9 x 16 MFMAs per wave and no per-tap barrier or weight reload
// remains.  One block per CU (72 KB weights + 2 x 44 KB halos = 160 KB of LDS); the epilogue uses the
// current halo buffer as its scratch tile.
constexpr int kT64 = 512;                             // 8 waves: 2 per SIMD to hide LDS / MFMA latency
template <bool PIPE>
__global__ __launch_bounds__(kT64, 1) void k_hconv64(HconvArgs a) {
  constexpr int HG = 44, HU = (HG + 7) / 8, HB = HG * 1024;   // (TH + 2) * (W + 2) <= 352 halo pixels
  constexpr int WB = 9 * 64 * 128;                      // 72 KB weights + 2 x 44 KB halos = 160 KB
  constexpr int RS = 64 * 2 + 16;
  static_assert(256 * RS + 2 * 8 * 64 * 4 <= HB, "epilogue scratch must fit one halo buffer");
  __shared__ __attribute__((aligned(16))) char smem[WB + 2 * HB];
  char* wimg = smem;
  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);   // w wave-uniform
  const int ntile = a.Bn * a.rtiles, HW2 = a.W + 2;
  const int lrow = glds_row(l), ch = glds_chunk(l, w & 1);
  const rsrc_t ar = make_rsrc(a.A, a.a_bytes), wr = make_rsrc(a.Wg, a.w_bytes);
  if ((int)blockIdx.x >= ntile) return;

  // weights: 72 one-KB groups (tap k = g / 8, rows n = 8 (g % 8) + lrow), 9 per wave
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int g = w + 8 * j, k = g >> 3, wi = a.tap[k] >> 16;
    glds16(wr, wimg + g * 1024, (uint32_t)((((g & 7) * 8 + lrow) * 9 * 64 + wi * 64 + ch * 8) * 2));
  }
  // halo pixel (hy, hx) of this lane's row in group w + 4u: fixed for every tile
  int hyx[HU];
#pragma unroll
  for (int u = 0; u < HU; ++u) {
    const int hr = 8 * (w + 8 * u) + (l >> 3), hy = hr / HW2;
    hyx[u] = (hy << 16) | (hr - hy * HW2);
  }
  auto issue_halo = [&](int tile, int buf) {
    const int b = tile / a.rtiles, oh0 = (tile - b * a.rtiles) * a.TH;
    char* h = smem + WB + buf * HB;
#pragma unroll
    for (int u = 0; u < HU; ++u) {
      const int hy = hyx[u] >> 16, hx = hyx[u] & 0xffff, ih = oh0 - 1 + hy, iw = hx - 1;
      const bool ok = hy < a.TH + 2 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
      if (w + 8 * u < HG)
        glds16(ar, h + (w + 8 * u) * 1024,
               ok ? (uint32_t)((((b * a.H + ih) * a.W + iw) * 64 + halo_dma_chunk(l, w & 1) * 8) * 2) : kOOB);
    }
  };

  const int wm = w, lr = l & 31, lh = l >> 5;            // 8 x 1 waves of 32 x 64
  const bool bnb = a.bnb.X != nullptr;
  BnbAcc za;                                           // accumulates over all of the block's tiles
  if (bnb) za.init(a.bnb, (t & 7) * 8);                 // a thread's chunk is the same in every tile
  float st_acc = 0.f;                                  // fprop statistics, thread t < 128: (t >> 6, t & 63)
  issue_halo(blockIdx.x, 0);
  int it = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x, ++it) {
    const int buf = it & 1;
    const int b = tile / a.rtiles, oh0 = (tile - b * a.rtiles) * a.TH;
    const int rows = min(a.TH, a.H - oh0), npx = rows * a.W;
    wait_vm<0>();                                      // this tile's halo (and the weights) landed
    __builtin_amdgcn_s_barrier();                      // ... for every wave; the other buffer is free
    // the epilogue's second input (residual gradient or BN input, never both) for this tile: issued
    // before the next halo's DMA and consumed after the MFMAs, so it lands under them (one CU streams
    // ~25 GB/s: a 32 KB tile read in the epilogue itself stalled the block ~1.3 us per tile)
    const size_t obase = ((size_t)b * a.H + oh0) * a.W;
    const bf16_t* pf = bnb ? a.bnb.X : a.R;
    uint4 pre[4];
    if (pf) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int c = t + kT64 * u, row = min(c >> 3, npx - 1);
        pre[u] = *reinterpret_cast<const uint4*>(pf + (obase + row) * 64 + (c & 7) * 8);
      }
    }
    if (tile + (int)gridDim.x < ntile) issue_halo(tile + gridDim.x, buf ^ 1);
    const char* halo = smem + WB + buf * HB;
    int hbase[1];
    {
      int p = wm * 32 + lr;
      p = p < npx ? p : 0;
      const int py = p / a.W, px = p - py * a.W;
      hbase[0] = (py + 1) * HW2 + px + 1;
    }
    f32x16 acc[1][2];
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[0][j] = f32x16{0.f};
    if constexpr (PIPE) {
      // a tap's 12 fragments (4 A from the halo, 8 B from the resident weights) are read before its
      // 8 MFMAs, so the reads of a tap overlap instead of each MFMA waiting on the read just issued
#pragma unroll
      for (int tp = 0; tp < 9; ++tp) {
        const int pk = a.tap[tp];
        const int td = (int)(signed char)(pk & 0xff) * HW2 + (int)(signed char)((pk >> 8) & 0xff);
        const char* Bi = wimg + tp * 8192;
        bf16x8 fa[4], fb[4][2];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          fa[s4] = halo_frag(halo, hbase[0] + td, 2 * s4 + lh);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[s4][j] = row_frag(Bi, j * 32 + lr, 2 * s4 + lh);
        }
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[0][j] = mfma_bf16(fa[s4], fb[s4][j], acc[0][j]);
      }
    } else {
      for (int tp = 0; tp < 9; ++tp) {
        const int pk = a.tap[tp];
        const int td = (int)(signed char)(pk & 0xff) * HW2 + (int)(signed char)((pk >> 8) & 0xff);
        const char* Bi = wimg + tp * 8192;
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          bf16x8 fa, fb[2];
          fa = halo_frag(halo, hbase[0] + td, 2 * s4 + lh);
#pragma unroll
          for (int j = 0; j < 2; ++j) fb[j] = row_frag(Bi, j * 32 + lr, 2 * s4 + lh);
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[0][j] = mfma_bf16(fa, fb[j], acc[0][j]);
        }
      }
    }
    __syncthreads();                                   // every wave is done reading this halo
    char* ot = smem + WB + buf * HB;                   // epilogue scratch: this tile's halo buffer
    float* sst = reinterpret_cast<float*>(ot + 256 * RS);   // [8][2][64]
    {
      const int i = 0;
      // statistics only when requested (fprop; the dgrad launches have none) and the row mask only on
      // the waves whose 32 rows run past npx (wave 7 at W = 56: 224 of 256 rows): both branches are
      // wave-uniform, so neither costs VALU where it does not apply
      const bool wfull = wm * 32 + 32 <= npx;
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int n = j * 32 + lr;
        bf16_t hv[16];
#pragma unroll
        for (int q = 0; q < 16; ++q) {
          const int m = wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
          hv[q] = f2bf(acc[i][j][q]);
          *reinterpret_cast<bf16_t*>(ot + m * RS + n * 2) = hv[q];
        }
        if (a.stats) {
          float s1 = 0.f, s2 = 0.f;
          if (wfull) {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              const float fv = bf2f(hv[q]);
              s1 += fv;
              s2 += fv * fv;
            }
          } else {
#pragma unroll
            for (int q = 0; q < 16; ++q) {
              const int m = wm * 32 + (q & 3) + 8 * (q >> 2) + 4 * lh;
              const float fv = m < npx ? bf2f(hv[q]) : 0.f;
              s1 += fv;
              s2 += fv * fv;
            }
          }
          s1 += __shfl_xor(s1, 32, 64);
          s2 += __shfl_xor(s2, 32, 64);
          if (lh == 0) { sst[(wm * 2 + 0) * 64 + n] = s1; sst[(wm * 2 + 1) * 64 + n] = s2; }
        }
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 4; ++u) {                      // 256 rows x 8 chunks of 16 B
      const int c = t + kT64 * u, row = c >> 3, cc = c & 7;
      if (row < npx) {
        uint4 v = *reinterpret_cast<const uint4*>(ot + row * RS + cc * 16);
        const size_t o = (obase + row) * 64 + cc * 8;
        if (a.R) {
          float f[8], r[8];
          unpack8(v, f);
          unpack8(pre[u], r);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] += r[e];
          v = pack8(f);
        }
        *reinterpret_cast<uint4*>(a.Y + o) = v;
        if (bnb) za.add(v, pre[u]);
      }
    }
    if (a.stats && t < 128) {
      float sum = 0.f;
#pragma unroll
      for (int k = 0; k < 8; ++k) sum += sst[(k * 2 + (t >> 6)) * 64 + (t & 63)];
      st_acc += sum;
    }
  }
  // one partial row per BLOCK (its tiles summed in a fixed order): <= #CUs rows, so the BN finalize
  // reads them directly (no k_fold_rows pass over one row per tile, thousands at B = 256)
  if (a.stats && t < 128) a.stats[((size_t)blockIdx.x * 2 + (t >> 6)) * 64 + (t & 63)] = st_acc;
  if (bnb) {
    __syncthreads();                                   // every wave is done with the last tile's LDS
    za.flush<8, 8, 64>(reinterpret_cast<float*>(smem + WB), a.bnb, (size_t)blockIdx.x, 64, 0);
  }
}

// ---- halo-tiled weight gradient, C = N = 64 (ResNet-18 layer1) ----
// dW[n][tap][c] = sum_p dY[p][n] X[p + d_tap][c]: the K dimension is the pixel, so both operands are
// read TRANSPOSED (ds_read_b64_tr_b16, K along image rows).  The implicit GEMM (k_wgrad) stages X once
// per tap column tile; here a persistent block walks row tiles (TH rows x W pixels, as k_hconv64),
// stages the tile's dY rows and its X halo once (double-buffered, both in the halo image layout), and
// accumulates all 9 taps x 64 c x 64 n in registers (4 waves x 9 32x32 tiles; a tap is a constant
// shift of the B rows); one fp32 slab per block, summed by k_wgrad_reduce.
__device__ __forceinline__ s4v tr_read_b64(uint32_t addr) {
  s4v v;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(v) : "v"(addr));
  return v;
}
// byte offset of the 8-byte piece (half hf) of 16-byte chunk ch in row r of a halo-layout image
__device__ __forceinline__ uint32_t hoffs(int r, int ch, int hf) {
  return (uint32_t)(r * 128 + 16 * (ch ^ hsw((r >> 1) & 7)) + 8 * hf);
}

struct HwgArgs {
  const bf16_t* dY;     // [Bn][H][W][64]
  const bf16_t* X;      // [Bn][H][W][64]
  float* part;          // [gridDim.x][64][9 * 64]
  uint32_t dy_bytes, x_bytes;
  int Bn, H, W, TH, rtiles;
  int tap[9];           // pack_tap(dh, dw, widx): column block widx gets shift (dh, dw)
};

constexpr int kHwgThreads = 576;                     // 9 waves: wave w owns tap w
__global__ __launch_bounds__(kHwgThreads, 1) void k_hwgrad64(HwgArgs a) {
  constexpr int NW = 9;
  constexpr int HG = 44, HB = HG * 1024;               // X halo: <= 352 rows
  constexpr int DG = 32, DB = DG * 1024;               // dY tile: 256 rows
  constexpr int BUF = HB + DB;
  __shared__ __attribute__((aligned(16))) char smem[2 * BUF];
  const int t = threadIdx.x, l = t & 63, w = __builtin_amdgcn_readfirstlane(t >> 6);   // w wave-uniform
  const int ntile = a.Bn * a.rtiles, HW2 = a.W + 2;
  const rsrc_t yr = make_rsrc(a.dY, a.dy_bytes), xr = make_rsrc(a.X, a.x_bytes);
  if ((int)blockIdx.x >= ntile) return;

  auto issue = [&](int tile, int buf) {
    const int b = tile / a.rtiles, oh0 = (tile - b * a.rtiles) * a.TH;
    const int npx = min(a.TH, a.H - oh0) * a.W;
    const int pbase = (b * a.H + oh0) * a.W;
    char* h = smem + buf * BUF;
#pragma unroll
    for (int u = 0; u < (HG + NW - 1) / NW; ++u) {
      const int g = w + NW * u;
      if (g < HG) {
        const int hr = 8 * g + (l >> 3), hy = hr / HW2, hx = hr - hy * HW2;
        const int ih = oh0 - 1 + hy, iw = hx - 1;
        const bool ok = hy < a.TH + 2 && (unsigned)ih < (unsigned)a.H && (unsigned)iw < (unsigned)a.W;
        const int dch = halo_dma_chunk(l, g & 1);
        glds16(xr, h + g * 1024, ok ? (uint32_t)((((b * a.H + ih) * a.W + iw) * 64 + dch * 8) * 2) : kOOB);
      }
    }
#pragma unroll
    for (int u = 0; u < (DG + NW - 1) / NW; ++u) {
      const int g = w + NW * u;
      if (g < DG) {
        const int k = 8 * g + (l >> 3), dch = halo_dma_chunk(l, g & 1);
        glds16(yr, h + HB + g * 1024, k < npx ? (uint32_t)(((pbase + k) * 64 + dch * 8) * 2) : kOOB);
      }
    }
  };

  // wave w = tap w: D[n][(w, c)] over both 32-row n tiles and both 32-column c halves
  const int g4 = l >> 4, i16 = l & 15, q = i16 >> 2, p4 = i16 & 3, h2 = g4 >> 1;
  const int hf = p4 & 1, cpart = 2 * (g4 & 1) + (p4 >> 1);
  const int pk = a.tap[w];
  const int td = (int)(signed char)(pk & 0xff) * HW2 + (int)(signed char)((pk >> 8) & 0xff);
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{0.f};
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  // fragments of one k-step: A (dY rows k, n chunks) x 2 n tiles, B (halo rows r + td, c chunks) x 2 halves
  struct Fr {
    s4v a[2][2], b[2][2];
  };
  // this lane's two K rows advance by 16 pixels per k-step: their image column and halo row index
  // (py + 1) * (W + 2) + px + 1 are kept incrementally -- a column wrap moves the halo row by the two
  // padding columns -- so the loop has no division and no per-step multiply (v_mul_lo_u32 is a
  // quarter-rate op; the K loop was VALU-bound); rows past npx read a valid halo row (their dY is 0)
  int kk0 = 0, px0 = 0, px1 = 0, hr0 = 0, hr1 = 0;
  auto start = [&]() {
    kk0 = 4 * h2 + q;
    const int py0 = kk0 / a.W, k1 = kk0 + 8, py1 = k1 / a.W;
    px0 = kk0 - py0 * a.W;
    px1 = k1 - py1 * a.W;
    hr0 = (py0 + 1) * HW2 + px0 + 1;
    hr1 = (py1 + 1) * HW2 + px1 + 1;
  };
  auto advance = [&]() {
    kk0 += 16;
    px0 += 16; px1 += 16;
    hr0 += 16; hr1 += 16;
    while (px0 >= a.W) { px0 -= a.W; hr0 += 2; }
    while (px1 >= a.W) { px1 -= a.W; hr1 += 2; }
  };
  // dY (A) rows advance by exactly 16 per k-step, which leaves their swizzle unchanged: the four A
  // offsets are per-lane constants plus 2048 * ks
  uint32_t aoffs[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    aoffs[i][0] = hoffs(4 * h2 + q, 4 * i + cpart, hf);
    aoffs[i][1] = hoffs(4 * h2 + q + 8, 4 * i + cpart, hf);
  }
  auto load = [&](Fr& f, uint32_t hbase, uint32_t ybase, int npx) {
    const int k0 = kk0, k1 = kk0 + 8;
    const int r0 = (k0 < npx ? hr0 : HW2 + 1) + td;
    const int r1 = (k1 < npx ? hr1 : HW2 + 1) + td;
    const uint32_t ya = ybase + 128u * (uint32_t)(kk0 - 4 * h2 - q);     // 2048 * ks
    const uint32_t b0 = hbase + r0 * 128 + 8 * hf, b1 = hbase + r1 * 128 + 8 * hf;
    const int s0 = hsw((r0 >> 1) & 7), s1 = hsw((r1 >> 1) & 7);
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f.a[i][0] = tr_read_b64(ya + aoffs[i][0]);
      f.a[i][1] = tr_read_b64(ya + aoffs[i][1]);
      f.b[i][0] = tr_read_b64(b0 + 16 * ((4 * i + cpart) ^ s0));
      f.b[i][1] = tr_read_b64(b1 + 16 * ((4 * i + cpart) ^ s1));
    }
  };
  auto mma = [&](const Fr& f) {
    bf16x8 fa[2], fb[2];
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      fa[i][0] = f.a[i][0][0]; fa[i][1] = f.a[i][0][1]; fa[i][2] = f.a[i][0][2]; fa[i][3] = f.a[i][0][3];
      fa[i][4] = f.a[i][1][0]; fa[i][5] = f.a[i][1][1]; fa[i][6] = f.a[i][1][2]; fa[i][7] = f.a[i][1][3];
      fb[i][0] = f.b[i][0][0]; fb[i][1] = f.b[i][0][1]; fb[i][2] = f.b[i][0][2]; fb[i][3] = f.b[i][0][3];
      fb[i][4] = f.b[i][1][0]; fb[i][5] = f.b[i][1][1]; fb[i][6] = f.b[i][1][2]; fb[i][7] = f.b[i][1][3];
    }
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j) acc[i][j] = mfma_bf16(fa[i], fb[j], acc[i][j]);
  };

  issue(blockIdx.x, 0);
  int it = 0;
  for (int tile = blockIdx.x; tile < ntile; tile += gridDim.x, ++it) {
    const int buf = it & 1;
    const int b = tile / a.rtiles, oh0 = (tile - b * a.rtiles) * a.TH;
    const int npx = min(a.TH, a.H - oh0) * a.W;
    wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    if (tile + (int)gridDim.x < ntile) issue(tile + gridDim.x, buf ^ 1);
    const uint32_t hbase = lds0 + buf * BUF, ybase = hbase + HB;
    const int nks = (npx + 15) >> 4;
    // software pipeline: the 8 transposed reads of k-step ks+1 are in flight during ks's 4 MFMAs
    Fr f0, f1;
    start();
    load(f0, hbase, ybase, npx);
    for (int ks = 0; ks < nks; ks += 2) {
      if (ks + 1 < nks) {
        advance();
        load(f1, hbase, ybase, npx);
        asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
      } else {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      }
      __builtin_amdgcn_sched_barrier(0);
      mma(f0);
      if (ks + 1 < nks) {
        if (ks + 2 < nks) {
          advance();
          load(f0, hbase, ybase, npx);
          asm volatile("s_waitcnt lgkmcnt(8)" ::: "memory");
        } else {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        }
        __builtin_amdgcn_sched_barrier(0);
        mma(f1);
      }
    }
  }
  // D[n][col]: registers = rows n, lane column = c; this wave's tap w -> dW[n][w][c]
  float* out = a.part + (size_t)blockIdx.x * 64 * 576;
  const int lr = l & 31, wi = pk >> 16;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int col = wi * 64 + 32 * j + lr;
#pragma unroll
      for (int qq = 0; qq < 16; ++qq) {
        const int n = 32 * i + (qq & 3) + 8 * (qq >> 2) + 4 * (l >> 5);
        out[(size_t)n * 576 + col] = acc[i][j][qq];
      }
    }
}

// Geometry of the halo path for a stride-1 3x3 / pad-1 conv over [Bn][H][W] with C -> NC channels:
// fills TH / rtiles / ntiles and returns BM (0 = not eligible: the implicit GEMM runs instead)
int hconv_geom(int Bn, int H, int W, int C, int NC, int R, int S, int stride, int pad, int& TH, int& rtiles) {
  static const bool off = [] {
    const char* e = getenv("PDE_CONV_HALO");
    return e && e[0] == '0';
  }();
  if (off || stride != 1 || R != 3 || S != 3 || pad != 1 || C % 64 || NC % 64 || W < 14 || W > 64 || Bn < 1)
    return 0;
  const int BM = NC % 128 == 0 ? 128 : 256;
  TH = min(H, BM / W);
  if (TH < 1 || (TH + 2) * (W + 2) > 8 * (BM == 256 ? hconv_groups<256>() : hconv_groups<128>())) return 0;
  rtiles = (H + TH - 1) / TH;
  return BM;
}

// k_hconv64 (persistent, C = NC = 64) runs this geometry: returns its grid (one block per CU, at most
// one per row tile), else 0.  Its statistics / BN-backward partials are one row per block.
int hconv64_grid(int Bn, int H, int W, int CA, int NC) {
  static const bool persistent = [] {
    const char* e = getenv("PDE_CONV_HALO_PERSIST");
    return !(e && e[0] == '0');
  }();
  int TH = 0, rtiles = 0;
  const int BM = hconv_geom(Bn, H, W, CA, NC, 3, 3, 1, 1, TH, rtiles);
  if (!(BM == 256 && CA == 64 && NC == 64 && (TH + 2) * (W + 2) <= 8 * 44 && persistent)) return 0;   // 44 used
  int ncu = 256, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess || ncu < 1)
    ncu = 256;
  return min(Bn * rtiles, ncu);
}

// partial rows (statistics or BN-backward) a halo-path launch writes: one per block of k_hconv64, one
// per row tile of k_hconv
int hconv_part_rows(int Bn, int H, int W, int CA, int NC) {
  const int g = hconv64_grid(Bn, H, W, CA, NC);
  if (g) return g;
  int TH = 0, rtiles = 0;
  return hconv_geom(Bn, H, W, CA, NC, 3, 3, 1, 1, TH, rtiles) ? Bn * rtiles : 0;
}

hipError_t launch_hconv(const void* A, const void* Wm, void* Y, const void* R, float* stats, int Bn, int H, int W,
                        int CA, int NC, const int* taps, hipStream_t st, const BnbArgs* bnb = nullptr) {
  HconvArgs a{};
  int TH = 0, rtiles = 0;
  const int BM = hconv_geom(Bn, H, W, CA, NC, 3, 3, 1, 1, TH, rtiles);
  if (!BM) return hipErrorInvalidValue;
  a.A = (const bf16_t*)A;
  a.Wg = (const bf16_t*)Wm;
  a.Y = (bf16_t*)Y;
  a.R = (const bf16_t*)R;
  a.stats = stats;
  if (bnb) a.bnb = *bnb;
  a.a_bytes = (uint32_t)((size_t)Bn * H * W * CA * 2);
  a.w_bytes = (uint32_t)((size_t)NC * 9 * CA * 2);
  a.Bn = Bn; a.H = H; a.W = W; a.CA = CA; a.NC = NC;
  a.TH = TH; a.rtiles = rtiles;
  for (int k = 0; k < 9; ++k) a.tap[k] = taps[k];
  if (const int g64 = hconv64_grid(Bn, H, W, CA, NC)) {
    a.ntiles = 1;
    const char* env = getenv("PDE_HC64_PIPE");   // 0: fragment reads interleaved with the MFMAs (A/B)
    if (env && atoi(env) == 0)
      hipLaunchKernelGGL(k_hconv64<false>, dim3(g64), dim3(kT64), 0, st, a);
    else
      hipLaunchKernelGGL(k_hconv64<true>, dim3(g64), dim3(kT64), 0, st, a);
  } else {
    const char* env = getenv("PDE_HCONV_V");   // tap-loop form (A/B): 0 hoisted addresses, 1 per tap
    const int v = env ? atoi(env) : 1;
    a.ntiles = NC / (BM == 256 ? 64 : 128);
    const dim3 grid(Bn * rtiles * a.ntiles);
    if (BM == 256)
      hipLaunchKernelGGL((v == 0 ? k_hconv<256, 64, 0> : k_hconv<256, 64, 1>), grid, dim3(kThreads), 0, st, a);
    else
      hipLaunchKernelGGL((v == 0 ? k_hconv<128, 128, 0> : k_hconv<128, 128, 1>), grid, dim3(kThreads), 0, st, a);
  }
  return hipGetLastError();
}

// dW (bf16) = sum over splits of the fp32 slabs [splits][n].  A 256-thread block = SL split lanes x
// 256/SL output lanes of 4 elements: the split range is walked by SL lanes in parallel (two slabs in
// flight each) and folded through LDS, so a small weight with hundreds of splits (1x1 downsample:
// 8192 outputs x ~200 slabs) is not one serial 200-load chain per thread on a handful of blocks.
template <int SL>
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ part, int splits, int64_t n,
                                                      bf16_t* __restrict__ dw) {
  constexpr int OL = 256 / SL;
  __shared__ float4 sh[SL][OL];
  const int ol = threadIdx.x % OL, sl = threadIdx.x / OL;
  const int64_t i = (blockIdx.x * (int64_t)OL + ol) * 4;
  float4 s = make_float4(0.f, 0.f, 0.f, 0.f);
  if (i < n) {
    int k = sl;
    for (; k + SL < splits; k += 2 * SL) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)k * n + i);
      const float4 w = *reinterpret_cast<const float4*>(part + (size_t)(k + SL) * n + i);
      s.x += v.x + w.x; s.y += v.y + w.y; s.z += v.z + w.z; s.w += v.w + w.w;
    }
    if (k < splits) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)k * n + i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  if constexpr (SL > 1) {
    sh[sl][ol] = s;
    __syncthreads();
    if (sl != 0) return;
#pragma unroll
    for (int j = 1; j < SL; ++j) {
      const float4 v = sh[j][ol];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  if (i >= n) return;
  const float f[4] = {s.x, s.y, s.z, s.w};
  *reinterpret_cast<uint2*>(dw + i) = pack4(f);
}

hipError_t launch_wgrad_reduce(const float* part, int splits, int64_t n, bf16_t* dw, hipStream_t st) {
  const int64_t n4 = n / 4;
  if (splits >= 32)
    hipLaunchKernelGGL(k_wgrad_reduce<16>, dim3((unsigned)((n4 + 15) / 16)), dim3(256), 0, st, part, splits, n, dw);
  else if (splits >= 4)
    hipLaunchKernelGGL(k_wgrad_reduce<4>, dim3((unsigned)((n4 + 63) / 64)), dim3(256), 0, st, part, splits, n, dw);
  else
    hipLaunchKernelGGL(k_wgrad_reduce<1>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, st, part, splits, n, dw);
  return hipGetLastError();
}

int g_conv_nst = 2;    // LDS pipeline depth of the conv kernels (2 or 3), pde_conv_set_stages

template <int BM, int BN>
hipError_t launch_igemm(IgemmArgs& a, hipStream_t st) {
  int maxm = 0;
  for (int z = 0; z < a.nphase; ++z) maxm = max(maxm, a.Bn * a.phase[z].Hq * a.phase[z].Wq);
  a.mtiles = (maxm + BM - 1) / BM;
  a.ntiles = a.NC / BN;
  const int grid = a.nphase * a.mtiles * a.ntiles;
  if (g_conv_nst == 2) hipLaunchKernelGGL((k_igemm<BM, BN, 2>), dim3(grid), dim3(kThreads), 0, st, a);
  else hipLaunchKernelGGL((k_igemm<BM, BN, 3>), dim3(grid), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

hipError_t dispatch_igemm(IgemmArgs& a, hipStream_t st) {
  if (a.NC % 128 == 0) return launch_igemm<128, 128>(a, st);
  return launch_igemm<256, 64>(a, st);
}

}  // namespace

extern "C" {

void pde_conv_set_stages(int nst) { g_conv_nst = nst == 3 ? 3 : 2; }

int pde_conv_fprop_mtiles(int M, int N) { return N % 128 == 0 ? (M + 127) / 128 : (M + 255) / 256; }

// rows of BN-statistics partials an fprop writes: one per M tile of whichever kernel runs it
int pde_conv_stats_rows(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int OH, int OW) {
  int TH = 0, rtiles = 0;
  if (hconv_geom(Bn, H, W, C, N, R, S, stride, pad, TH, rtiles)) return hconv_part_rows(Bn, H, W, C, N);
  return pde_conv_fprop_mtiles(Bn * OH * OW, N);
}

hipError_t pde_conv_fprop(const void* x, const void* w, void* y, float* stats, int Bn, int H, int W, int C, int N,
                          int R, int S, int stride, int pad, int OH, int OW, hipStream_t st) {
  if (C % 64 || N % 64 || R * S > 9) return hipErrorInvalidValue;
  {
    int TH = 0, rtiles = 0;
    if (hconv_geom(Bn, H, W, C, N, R, S, stride, pad, TH, rtiles)) {
      int taps[9];
      for (int k = 0; k < 9; ++k) taps[k] = pack_tap(k / 3 - 1, k % 3 - 1, k);
      return launch_hconv(x, w, y, nullptr, stats, Bn, H, W, C, N, taps, st);
    }
  }
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
  P.inv_hw = 1.0f / (float)(OH * OW);
  P.inv_w = 1.0f / (float)OW;
  for (int r = 0; r < R; ++r)
    for (int s = 0; s < S; ++s) {
      const int k = r * S + s;
      P.tap[k] = pack_tap(r - pad, s - pad, k);
    }
  return dispatch_igemm(a, st);
}

hipError_t pde_conv_wtrans(const void* w, void* wt, int N, int T, int C, hipStream_t st) {
  if (N % 64 || C % 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wtrans, dim3(C / 64, N / 64, T), dim3(256), 0, st, (const bf16_t*)w, (bf16_t*)wt, N, T, C);
  return hipGetLastError();
}

// desc: device array of nconv WtDesc (tile0 = running sum of (C/64)*(N/64)*T); total = all tiles
hipError_t pde_conv_wtrans_batch(const void* desc, int nconv, int total, long long* ctr, int ncnt, hipStream_t st) {
  if (ncnt > 256) return hipErrorInvalidValue;
  if (nconv < 1 || total < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_wtrans_batch, dim3(total), dim3(256), 0, st, (const WtDesc*)desc, nconv, ctr, ncnt);
  return hipGetLastError();
}
int pde_conv_wtdesc_bytes() { return (int)sizeof(WtDesc); }

// dX (NHWC [Bn][H][W][C]) from dY ([Bn][OH][OW][N]) and Wt = [C][R*S][N] (pde_conv_wtrans);
// res (optional, NHWC like dX): dX = dgrad + res -- the residual / second-consumer gradient of the
// conv input accumulated in the epilogue instead of a separate add pass
// dy2 / wt2 (optional): a 1x1 / stride-2 / pad-0 convolution of the same input with the same output
// shape (a ResNet downsample) whose input gradient is accumulated in the same pass: its dy2 [Bn][OH][OW][N]
// and transposed weights wt2 [C][1][N] are K stages of the (0, 0) phase (the only input pixels it reads)
// rows of BN-backward partials a stride-1 dgrad with `bnb` writes: one per M tile of its kernel
int pde_conv_dgrad_bnb_rows(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad) {
  if (stride != 1) return 0;
  int TH = 0, rtiles = 0;
  if (hconv_geom(Bn, H, W, N, C, R, S, stride, pad, TH, rtiles)) return hconv_part_rows(Bn, H, W, N, C);
  return pde_conv_fprop_mtiles(Bn * H * W, C);
}

// bx / bsc / bsh / bmu / brs / bpart (optional, bx != nullptr; stride 1 only): BN-backward partials
// of dX for a BN + ReLU whose input was bx (BnbArgs), into bpart[pde_conv_dgrad_bnb_rows][2][C]
hipError_t pde_conv_dgrad(const void* dy, const void* wt, void* dx, const void* res, const void* dy2, const void* wt2,
                          int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int OH, int OW,
                          const void* bx, const float* bsc, const float* bsh, const float* bmu, const float* brs,
                          float* bpart, hipStream_t st) {
  if (C % 64 || N % 64 || R * S > 9 || stride < 1 || stride > 2) return hipErrorInvalidValue;
  if (dy2 && (stride != 2 || !wt2 || (H - 1) / 2 + 1 != OH || (W - 1) / 2 + 1 != OW)) return hipErrorInvalidValue;
  BnbArgs z{(const bf16_t*)bx, bsc, bsh, bmu, brs, bpart};
  // (the epilogue prefetches one second input: the residual gradient or the BN input, not both)
  if (bx && (stride != 1 || dy2 || res || !bsc || !bsh || !bmu || !brs || !bpart)) return hipErrorInvalidValue;
  {
    // stride-1 3x3 / pad-1: the input gradient is the flipped-tap conv of dy with Wt (halo path)
    int TH = 0, rtiles = 0;
    if (!dy2 && OH == H && OW == W && hconv_geom(Bn, H, W, N, C, R, S, stride, pad, TH, rtiles)) {
      int taps[9];
      for (int k = 0; k < 9; ++k) taps[k] = pack_tap(1 - k / 3, 1 - k % 3, k);
      return launch_hconv(dy, wt, dx, res, nullptr, Bn, H, W, N, C, taps, st, bx ? &z : nullptr);
    }
  }
  IgemmArgs a{};
  if (bx) a.bnb = z;
  a.A = (const bf16_t*)dy;
  a.W = (const bf16_t*)wt;
  a.Y = (bf16_t*)dx;
  a.R = (const bf16_t*)res;
  a.A2 = (const bf16_t*)dy2;
  a.W2 = (const bf16_t*)wt2;
  a.a2_bytes = dy2 ? (uint32_t)((size_t)Bn * OH * OW * N * 2) : 0u;
  a.w2_bytes = dy2 ? (uint32_t)((size_t)N * C * 2) : 0u;
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
    P.inv_hw = 1.0f / (float)(P.Hq * P.Wq);
    P.inv_w = 1.0f / (float)P.Wq;
    P.ntap = 0;
    P.ntap2 = (dy2 && z == 0) ? 1 : 0;
    for (int r = 0; r < R; ++r) {
      const int nh = P.ph + pad - r;
      if (((nh % stride) + stride) % stride) continue;
      for (int s = 0; s < S; ++s) {
        const int nw = P.pw + pad - s;
        if (((nw % stride) + stride) % stride) continue;
        const int k = P.ntap++;
        // floor division of (possibly negative) exact multiples of stride
        P.tap[k] = pack_tap(nh >= 0 ? nh / stride : -((-nh) / stride), nw >= 0 ? nw / stride : -((-nw) / stride),
                            r * S + s);
      }
    }
  }
  return dispatch_igemm(a, st);
}

// halo-tiled layer1 wgrad (k_hwgrad64): row tiles as k_hconv64; returns the persistent grid (= slabs)
// or 0 when not eligible
static int hwgrad_grid(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int& TH, int& rtiles) {
  static const bool off = [] {
    const char* e = getenv("PDE_CONV_HALO_WGRAD");
    return e && e[0] == '0';
  }();
  if (off || C != 64 || N != 64 || R != 3 || S != 3 || stride != 1 || pad != 1 || W < 14 || W > 64) return 0;
  TH = min(H, 256 / W);
  if (TH < 1 || (TH + 2) * (W + 2) > 352) return 0;
  rtiles = (H + TH - 1) / TH;
  int ncu = 256, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
    ncu = 256;
  return min(Bn * rtiles, ncu);
}

int pde_conv_wgrad_splits2(int Bn, int H, int W, int C, int N, int R, int S, int stride, int pad, int OH, int OW) {
  int TH = 0, rtiles = 0;
  const int g = hwgrad_grid(Bn, H, W, C, N, R, S, stride, pad, TH, rtiles);
  return g ? g : pde_conv_wgrad_splits(Bn, OH, OW, N, R * S, C);
}

int pde_conv_wgrad_splits(int Bn, int OH, int OW, int N, int T, int C) {
  // At most one round of co-resident blocks (2 per CU) and >= 16 pixel stages per block: enough
  // parallelism without making the fp32 slab round trip (splits x N x T*C x 4 B, written and re-read)
  // dominate.  Rounded DOWN: the former ceil(512 / tiles) launched 513-576 blocks for the 3x3 convs of
  // layers 2-4, and the few blocks past the first round ran as a tail of a whole block's duration
  // (tools/conv_bench.py --wgrad-blocks: l3 3x3 109.5 -> 76.7 us, l2.0 conv1 72.7 -> 50.4 us;
  // profiles/r3_models/wgrad_blocks_sweep.jsonl).
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess ||
      hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu < 1)
    ncu = 256;
  const int P = Bn * OH * OW, stages = (P + 63) / 64;
  const int BM = N % 128 == 0 ? 128 : 64, BN = 128;
  const int tiles = (N / BM) * ((T * C + BN - 1) / BN);
  int splits = 2 * ncu / tiles;
  splits = min(splits, stages / 16);
  return max(1, splits);
}

// out (bf16) = sum over S fp32 slabs [S][n] (split-K partial products), n % 4 == 0
hipError_t pde_sum_slabs_bf16(const float* part, int S, int64_t n, void* out, hipStream_t st) {
  if (n % 4 || S < 1) return hipErrorInvalidValue;
  return launch_wgrad_reduce(part, S, n, (bf16_t*)out, st);
}

// part: fp32 [splits][N][T*C] scratch; dw: bf16 [N][T*C]
hipError_t pde_conv_wgrad(const void* dy, const void* x, float* part, int splits, void* dw, int Bn, int H, int W,
                          int C, int N, int R, int S, int stride, int pad, int OH, int OW, hipStream_t st) {
  if (C % 64 || N % 64 || splits < 1) return hipErrorInvalidValue;
  {
    int TH = 0, rtiles = 0;
    const int g = hwgrad_grid(Bn, H, W, C, N, R, S, stride, pad, TH, rtiles);
    if (g && g == splits) {
      HwgArgs h{};
      h.dY = (const bf16_t*)dy;
      h.X = (const bf16_t*)x;
      h.part = part;
      h.dy_bytes = (uint32_t)((size_t)Bn * H * W * 64 * 2);
      h.x_bytes = h.dy_bytes;
      h.Bn = Bn; h.H = H; h.W = W; h.TH = TH; h.rtiles = rtiles;
      for (int k = 0; k < 9; ++k) h.tap[k] = pack_tap(k / 3 - 1, k % 3 - 1, k);
      hipLaunchKernelGGL(k_hwgrad64, dim3(g), dim3(kHwgThreads), 0, st, h);
      PDE_HIP_CHECK(hipGetLastError());
      return launch_wgrad_reduce(part, splits, (int64_t)N * 9 * C, (bf16_t*)dw, st);
    }
  }
  WgradArgs a{};
  a.dY = (const bf16_t*)dy;
  a.X = (const bf16_t*)x;
  a.part = part;
  a.dy_bytes = (uint32_t)((size_t)Bn * OH * OW * N * 2);
  a.x_bytes = (uint32_t)((size_t)Bn * H * W * C * 2);
  a.Bn = Bn; a.IH = H; a.IW = W; a.C = C; a.OH = OH; a.OW = OW; a.N = N; a.S = S;
  a.stride = stride; a.pad = pad; a.T = R * S;
  a.P = Bn * OH * OW;
  a.inv_hw = 1.0f / (float)(OH * OW);
  a.inv_w = 1.0f / (float)OW;
  {
    static const int incr_env = [] {   // PDE_WGRAD_INCR=0: per-stage divisions instead of the row walk
      const char* e = getenv("PDE_WGRAD_INCR");
      return e == nullptr ? 1 : atoi(e) != 0;
    }();
    a.incr = (64 / OW + 1 < 2 * OH) ? incr_env : 0;   // <= 2 carries of oh into b per 64-pixel step
  }
  const int stages = (a.P + 63) / 64;
  a.stages_per_split = (stages + splits - 1) / splits;
  const int TC = a.T * C;
  const bool inc = a.incr != 0;
  if (N % 128 == 0) {
    a.mtiles = N / 128; a.ntiles = (TC + 127) / 128;
    const dim3 grid(splits * a.mtiles * a.ntiles);
    if (g_conv_nst == 2)
      hipLaunchKernelGGL((inc ? k_wgrad<128, 128, 2, true> : k_wgrad<128, 128, 2, false>), grid, dim3(kThreads), 0, st, a);
    else
      hipLaunchKernelGGL((inc ? k_wgrad<128, 128, 3, true> : k_wgrad<128, 128, 3, false>), grid, dim3(kThreads), 0, st, a);
  } else {
    a.mtiles = N / 64; a.ntiles = (TC + 127) / 128;
    const dim3 grid(splits * a.mtiles * a.ntiles);
    if (g_conv_nst == 2)
      hipLaunchKernelGGL((inc ? k_wgrad<64, 128, 2, true> : k_wgrad<64, 128, 2, false>), grid, dim3(kThreads), 0, st, a);
    else
      hipLaunchKernelGGL((inc ? k_wgrad<64, 128, 3, true> : k_wgrad<64, 128, 3, false>), grid, dim3(kThreads), 0, st, a);
  }
  PDE_HIP_CHECK(hipGetLastError());
  const int64_t n = (int64_t)N * TC;
  return launch_wgrad_reduce(part, splits, n, (bf16_t*)dw, st);
}

}  // extern "C"
