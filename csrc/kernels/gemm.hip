// bf16 MFMA GEMM with fused epilogues for the GPT-2 config of BASELINE.json (the nn.Linear op
// class of /root/reference/mnist/main.py:136-137, at GPT-2 shapes): fprop, dgrad and split-K
// wgrad of every projection and of the tied LM head, on v_mfma_f32_32x32x16_bf16, fp32 accumulate.
//
//   C[m][n] = sum_k A(m, k) * B(k, n)      (N, and M / K where staged in chunks, multiples of 8;
//                                          ragged tiles and the K % 64 tail are masked)
//   A(m, k) = A[m * lda + k]  (TA = 0: K-contiguous rows)   or  A[k * lda + m]  (TA = 1)
//   B(k, n) = B[n * ldb + k]  (TB = 0: nn.Linear weight)    or  B[k * ldb + n]  (TB = 1)
//
//   fprop  Y[tok][out]  = X[tok][in] . W[out][in]^T        TA = 0, TB = 0  (+ bias, + GELU)
//   dgrad  dX[tok][in]  = dY[tok][out] . W[out][in]        TA = 0, TB = 1  (+ GELU backward)
//   wgrad  dW[out][in]  = dY[tok][out]^T . X[tok][in]      TA = 1, TB = 1  (+ bias gradient)
//
// Block tile BM x BN = (WM*TM*32) x (WN*TN*32), WM*WN waves, each owning TM x TN 32x32 accumulators.
// K is staged 64 deep through NST LDS buffers filled by LDS-DMA (buffer_load ... lds, 16 B per
// lane): a K-contiguous operand is a [rows][64] image, a transposed operand a set of [64 k][64]
// images, both in the XOR-swizzled 128-byte-row layout of pde_lds.h, so row operands are read with
// conflict-free ds_read_b128 and transposed ones with ds_read_b64_tr_b16 -- no operand is ever
// transposed in memory.  Pipeline per stage: counted vmcnt (this wave's DMA of the stage, the
// younger stage stays in flight) -> raw s_barrier -> issue the stage NST-1 ahead -> 4 k-steps of
// MFMAs with the next k-step's fragments read while the current one computes.  All LDS reads are
// inline asm with immediate offsets (two lane bases per operand), so hipcc neither spends VALU on
// LDS addresses nor inserts a vmcnt(0) drain for the in-flight DMA in front of them.
//
// The MFMA is issued with the operands swapped (D' = B^T A^T), so a lane's accumulator registers
// hold FOUR CONSECUTIVE COLUMNS of C: the epilogue writes 8-byte pieces into an LDS tile and stores
// C as coalesced 16-byte rows, applying bias (fp32, before the single bf16 rounding), GELU (writing
// pre-activation and activation), or the GELU backward (reading the saved pre-activation).
//
// Bias gradient: db[m] = sum_k A(m, k) is one more MFMA per k-step against a ones fragment, issued
// only by the blocks of the first column tile (k-steps shared round-robin by their WN waves), into
// fp32 partials [split][M] that the split-K reduction kernel folds together with dW.
//
// Blocks: XCD-aware id remap (pde_hip.h), then groups of 8 row tiles x all column tiles so the
// blocks sharing an XCD's L2 share operand rows; split-K slices of one tile are adjacent ids.
#include <type_traits>

#include "pde_act.h"
#include "pde_bf16.h"
#include "pde_hip.h"
#include "pde_kernels.h"
#include "pde_lds.h"

namespace {

using namespace pde_lds;

enum Epi { kBf16 = 0, kGelu = 1, kGeluBwd = 2, kSlab = 3 };

struct GemmArgs {
  const bf16_t* A;
  const bf16_t* B;
  void* C;               // bf16 [M][ldc], or fp32 slabs [splits][M][ldc] (kSlab)
  bf16_t* C2;            // kGelu: activation output [M][ldc] (C gets the pre-activation)
  const bf16_t* bias;    // [N] or null (kBf16 / kGelu)
  const bf16_t* aux;     // kGeluBwd: pre-activation [M][ldc]
  float* colsum;         // [splits][M] bias-gradient partials (CS) or null
  uint32_t a_bytes, b_bytes;
  int M, N, K, lda, ldb, ldc;
  int mtiles, ntiles, kper;
};

// Transposed-read lane bases delivering the STANDARD k order (element j of a lane in half h is
// k = 8h + j, as a ds_read_b128 row fragment): rows 8h + q and 8h + 4 + q of the k-step, so a
// transposed operand can meet a row-read operand in one MFMA.  (pde_lds.h's tr_lane_off reads rows
// 4h + q / 8 + 4h + q: consistent only with another transposed read.)  Same bank pattern: each
// 32-lane half still reads an aligned 4-row block per instruction.
__device__ __forceinline__ uint2 tr_lane_off_k8() {
  const int lane = threadIdx.x & 63, g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3, h = g >> 1;
  const int ch = 2 * (g & 1) + (p >> 1);
  return make_uint2(toff(8 * h + q, ch) + 8 * (p & 1), toff(8 * h + 4 + q, ch) + 8 * (p & 1));
}

template <int I, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    static_for<I + 1, N>(f);
  }
}

template <int OFF>
__device__ __forceinline__ bf16x8 rd128(uint32_t addr) {
  bf16x8 v;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(v) : "v"(addr), "n"(OFF));
  return v;
}

// lane bases of a row-operand fragment (rows r0 + lane&31, k-step chunk 2S + lane>>5): toff() of the
// even / odd k-steps; the k-step pair S>>1 is +512 and row block i is +4096 (32 rows)
__device__ __forceinline__ uint2 row_lane_off(int r0) {
  const int l = threadIdx.x & 63, row = r0 + (l & 31), h = l >> 5;
  return make_uint2(toff(row, h), toff(row, 2 + h));
}

template <int TM, int TN, int WM, int WN, int NST, bool TA, bool TB, int EPI, bool CS>
__global__ __launch_bounds__(64 * WM * WN, 1) void k_gemm(GemmArgs a) {
  constexpr int NW = WM * WN, NT = 64 * NW;
  constexpr int WTM = TM * 32, WTN = TN * 32, BM = WM * WTM, BN = WN * WTN;
  constexpr int ABYTES = BM * 128, BBYTES = BN * 128, STAGE = ABYTES + BBYTES;
  constexpr int AG = BM / 8 / NW, BG = BN / 8 / NW;   // LDS-DMA wave-instructions per wave per stage
  static_assert(AG * 8 * NW == BM && BG * 8 * NW == BN, "one 8-row group per wave-instruction");
  static_assert((!TA || BM % 64 == 0) && (!TB || BN % 64 == 0), "transposed operands come in 64-wide images");
  constexpr int LPS = AG + BG;
  constexpr int RS = BN * 2 + 16;                      // epilogue LDS tile row stride (bytes)
  constexpr int TILE_BYTES = EPI == kSlab ? 0 : BM * RS;
  constexpr int EPI_BYTES = TILE_BYTES + (CS ? WN * BM * 4 : 0);
  constexpr int SMEM = NST * STAGE > EPI_BYTES ? NST * STAGE : EPI_BYTES;
  __shared__ __attribute__((aligned(16))) char smem[SMEM];

  const int t = threadIdx.x, l = t & 63, lr = l & 31, lh = l >> 5;
  const int w = __builtin_amdgcn_readfirstlane(t >> 6);   // wave-uniform: scalar branches / addresses
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  const int ntile = a.mtiles * a.ntiles;
  const int split = id / ntile, rem = id - split * ntile;
  constexpr int G = 8;
  const int grp = rem / (G * a.ntiles), r2 = rem - grp * (G * a.ntiles);
  const int gsz = min(G, a.mtiles - grp * G);
  const int mt = grp * G + r2 % gsz, nt = r2 / gsz;
  const int m0 = mt * BM, n0 = nt * BN;
  const int kbeg = split * a.kper;
  const int KT = (min(a.K, kbeg + a.kper) - kbeg + 63) >> 6;   // K % 64 tail: see issue()
  const int wm = w / WN, wn = w % WN;

  // ---- LDS-DMA source offsets (bytes) of this wave's 8-row groups at stage 0 ----
  const int lrow = glds_row(l);
  uint32_t aoff[AG], boff[BG];
  int ach[AG], bch[BG];                                // k offset of this lane's 16-byte chunk
#pragma unroll
  for (int u = 0; u < AG; ++u) {
    const int g = NW * u + w, ch = glds_chunk(l, g & 1);
    ach[u] = 8 * ch;
    if constexpr (!TA) {
      const int m = m0 + 8 * g + lrow;
      aoff[u] = m < a.M ? (uint32_t)(((size_t)m * a.lda + kbeg + 8 * ch) * 2) : kOOB;
    } else {
      const int k = kbeg + 8 * (g & 7) + lrow, m = m0 + 64 * (g >> 3) + 8 * ch;
      aoff[u] = m < a.M ? (uint32_t)(((size_t)k * a.lda + m) * 2) : kOOB;
    }
  }
#pragma unroll
  for (int v = 0; v < BG; ++v) {
    const int g = NW * v + w, ch = glds_chunk(l, g & 1);
    bch[v] = 8 * ch;
    if constexpr (!TB) {
      const int n = n0 + 8 * g + lrow;
      boff[v] = n < a.N ? (uint32_t)(((size_t)n * a.ldb + kbeg + 8 * ch) * 2) : kOOB;
    } else {
      const int k = kbeg + 8 * (g & 7) + lrow, n = n0 + 64 * (g >> 3) + 8 * ch;
      boff[v] = n < a.N ? (uint32_t)(((size_t)k * a.ldb + n) * 2) : kOOB;
    }
  }
  const uint32_t astep = TA ? (uint32_t)a.lda * 128u : 128u, bstep = TB ? (uint32_t)a.ldb * 128u : 128u;
  const rsrc_t ar = make_rsrc(a.A, a.a_bytes), br = make_rsrc(a.B, a.b_bytes);
  // K tail (K % 64 != 0, K % 8 == 0): a K-contiguous operand's chunks past K read zeros; a
  // transposed operand's rows past K are past its buffer resource (a_bytes / b_bytes end at row K)
  auto issue = [&](int kt, int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + ABYTES;
    const int kb = kbeg + kt * 64;
#pragma unroll
    for (int u = 0; u < AG; ++u)
      glds16(ar, As + (NW * u + w) * 1024, (TA || kb + ach[u] < a.K) ? aoff[u] + (uint32_t)kt * astep : kOOB);
#pragma unroll
    for (int v = 0; v < BG; ++v)
      glds16(br, Bs + (NW * v + w) * 1024, (TB || kb + bch[v] < a.K) ? boff[v] + (uint32_t)kt * bstep : kOOB);
  };

  // ---- fragment lane bases (relative to a stage's A / B image) ----
  uint2 abase[TA ? TM : 1], bbase[TB ? TN : 1];
  if constexpr (TA) {
#pragma unroll
    for (int i = 0; i < TM; ++i) abase[i] = add2(tr_lane_off_k8(), colblk_off(wm * TM + i));
  } else {
    abase[0] = row_lane_off(wm * WTM);
  }
  if constexpr (TB) {
#pragma unroll
    for (int j = 0; j < TN; ++j) bbase[j] = add2(tr_lane_off_k8(), colblk_off(wn * TN + j));
  } else {
    bbase[0] = row_lane_off(wn * WTN);
  }
  const uint32_t lds0 = (uint32_t)(uintptr_t)(lds_char*)smem;

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x16{0.f};
  f32x16 accb[CS ? TM : 1];
#pragma unroll
  for (int i = 0; i < (CS ? TM : 1); ++i) accb[i] = f32x16{0.f};
  const bool cs_on = CS && a.colsum != nullptr && nt == 0;
  bf16x8 ones;
#pragma unroll
  for (int e = 0; e < 8; ++e) ones[e] = (short)0x3f80;

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
      const uint32_t sa = lds0 + buf * STAGE, sb = sa + ABYTES;
      uint2 ab[TA ? TM : 1], bb[TB ? TN : 1];
#pragma unroll
      for (int i = 0; i < (TA ? TM : 1); ++i) ab[i] = add2(abase[i], sa);
#pragma unroll
      for (int j = 0; j < (TB ? TN : 1); ++j) bb[j] = add2(bbase[j], sb);

      bf16x8 fa0[TM], fb0[TN], fa1[TM], fb1[TN];
      auto load = [&](auto S_, bf16x8* fa, bf16x8* fb) {
        constexpr int S = decltype(S_)::value;
        static_for<0, TM>([&](auto I_) {
          constexpr int i = decltype(I_)::value;
          if constexpr (TA) fa[i] = trpair<2048 * S>(ab[i]);
          else fa[i] = rd128<4096 * i + 512 * (S >> 1)>((S & 1) ? ab[0].y : ab[0].x);
        });
        static_for<0, TN>([&](auto J_) {
          constexpr int j = decltype(J_)::value;
          if constexpr (TB) fb[j] = trpair<2048 * S>(bb[j]);
          else fb[j] = rd128<4096 * j + 512 * (S >> 1)>((S & 1) ? bb[0].y : bb[0].x);
        });
      };
      auto mm = [&](auto S_, const bf16x8* fa, const bf16x8* fb) {
        constexpr int S = decltype(S_)::value;
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) acc[i][j] = mfma_bf16(fb[j], fa[i], acc[i][j]);
        if constexpr (CS) {
          if (cs_on && (S % WN) == wn) {
#pragma unroll
            for (int i = 0; i < TM; ++i) accb[i] = mfma_bf16(ones, fa[i], accb[i]);
          }
        }
      };
      using S0 = std::integral_constant<int, 0>;
      using S1 = std::integral_constant<int, 1>;
      using S2 = std::integral_constant<int, 2>;
      using S3 = std::integral_constant<int, 3>;
      load(S0{}, fa0, fb0);
      lgkm_fence();
      load(S1{}, fa1, fb1);
      mm(S0{}, fa0, fb0);
      lgkm_fence();
      load(S2{}, fa0, fb0);
      mm(S1{}, fa1, fb1);
      lgkm_fence();
      load(S3{}, fa1, fb1);
      mm(S2{}, fa0, fb0);
      lgkm_fence();
      mm(S3{}, fa1, fb1);
      buf = buf + 1 == NST ? 0 : buf + 1;
    }
  }
  __syncthreads();                                     // every wave is done reading the stage buffers

  // ---- epilogue.  Lane (lr, lh) of accumulator (i, j) holds C[row wm*WTM + 32i + lr]
  //      [col wn*WTN + 32j + 8g + 4lh + e] in register 4g + e ----
  if constexpr (EPI == kSlab) {
    float* out = reinterpret_cast<float*>(a.C) + (size_t)split * a.M * a.ldc;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int m = m0 + wm * WTM + 32 * i + lr;
      if (m < a.M) {
#pragma unroll
        for (int j = 0; j < TN; ++j)
#pragma unroll
          for (int g = 0; g < 4; ++g) {
            const int n = n0 + wn * WTN + 32 * j + 8 * g + 4 * lh;
            if (n < a.N)
              *reinterpret_cast<float4*>(out + (size_t)m * a.ldc + n) =
                  make_float4(acc[i][j][4 * g], acc[i][j][4 * g + 1], acc[i][j][4 * g + 2], acc[i][j][4 * g + 3]);
          }
      }
    }
  } else {
    const bool has_bias = (EPI == kBf16 || EPI == kGelu) && a.bias != nullptr;
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int nl = wn * WTN + 32 * j + 8 * g + 4 * lh;
        float bv[4] = {0.f, 0.f, 0.f, 0.f};
        if (has_bias && n0 + nl < a.N) unpack4(*reinterpret_cast<const uint2*>(a.bias + n0 + nl), bv);
#pragma unroll
        for (int i = 0; i < TM; ++i) {
          const int ml = wm * WTM + 32 * i + lr;
          const float v[4] = {acc[i][j][4 * g] + bv[0], acc[i][j][4 * g + 1] + bv[1], acc[i][j][4 * g + 2] + bv[2],
                              acc[i][j][4 * g + 3] + bv[3]};
          *reinterpret_cast<uint2*>(smem + ml * RS + nl * 2) = pack4(v);
        }
      }
  }
  if constexpr (CS) {
    if (cs_on && lh == 0) {
      float* csl = reinterpret_cast<float*>(smem + TILE_BYTES);
#pragma unroll
      for (int i = 0; i < TM; ++i) csl[wn * BM + wm * WTM + 32 * i + lr] = accb[i][0];
    }
  }
  if constexpr (EPI != kSlab || CS) __syncthreads();
  if constexpr (CS) {
    if (cs_on && t < BM && m0 + t < a.M) {
      const float* csl = reinterpret_cast<const float*>(smem + TILE_BYTES);
      float s = 0.f;
#pragma unroll
      for (int q = 0; q < WN; ++q) s += csl[q * BM + t];
      a.colsum[(size_t)split * a.M + m0 + t] = s;
    }
  }
  if constexpr (EPI != kSlab) {
    constexpr int CPR = BN / 8;                        // 16-byte chunks per tile row
    bf16_t* C = reinterpret_cast<bf16_t*>(a.C);
#pragma unroll 4
    for (int c = t; c < BM * CPR; c += NT) {
      const int row = c / CPR, cc = c - row * CPR;
      const int m = m0 + row, n = n0 + 8 * cc;
      if (m < a.M && n < a.N) {
        const uint4 v = *reinterpret_cast<const uint4*>(smem + row * RS + cc * 16);
        const size_t o = (size_t)m * a.ldc + n;
        if constexpr (EPI == kBf16) {
          *reinterpret_cast<uint4*>(C + o) = v;
        } else if constexpr (EPI == kGelu) {
          *reinterpret_cast<uint4*>(C + o) = v;
          float f[8];
          unpack8(v, f);
#pragma unroll
          for (int e = 0; e < 8; ++e) f[e] = gelu_t(f[e], nullptr);
          *reinterpret_cast<uint4*>(a.C2 + o) = pack8(f);
        } else {                                       // kGeluBwd: dX = bf16(acc) * gelu'(pre)
          float f[8], p[8];
          unpack8(v, f);
          unpack8(*reinterpret_cast<const uint4*>(a.aux + o), p);
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            float d;
            gelu_t(p[e], &d);
            f[e] *= d;
          }
          *reinterpret_cast<uint4*>(C + o) = pack8(f);
        }
      }
    }
  }
}

// dW (bf16 [M][N] contiguous) = sum of the fp32 slabs [S][M][N]; blocks past the dW range fold the
// bias-gradient partials [S][M] into db (bf16) the same way
__global__ __launch_bounds__(256) void k_gemm_reduce(const float* __restrict__ part, int S, int64_t mn,
                                                     bf16_t* __restrict__ dw, int nb_main, const float* __restrict__ cs,
                                                     int M, bf16_t* __restrict__ db) {
  if ((int)blockIdx.x < nb_main) {
    const int64_t i = (blockIdx.x * 256ll + threadIdx.x) * 4;
    if (i >= mn) return;
    float4 s = *reinterpret_cast<const float4*>(part + i);
    for (int k = 1; k < S; ++k) {
      const float4 v = *reinterpret_cast<const float4*>(part + (size_t)k * mn + i);
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
    const float f[4] = {s.x, s.y, s.z, s.w};
    *reinterpret_cast<uint2*>(dw + i) = pack4(f);
  } else {
    const int m = ((int)blockIdx.x - nb_main) * 256 + threadIdx.x;
    if (m >= M) return;
    float s = 0.f;
    for (int k = 0; k < S; ++k) s += cs[(size_t)k * M + m];
    db[m] = f2bf(s);
  }
}

// ---- tile configurations ----
//   0: 256 x 192, 8 waves (4 x 2) of 64 x 96, 2 stages (112 KB)
//   1: 256 x 128, 8 waves (4 x 2) of 64 x 64, 3 stages (144 KB)
//   2: 128 x 128, 4 waves (2 x 2) of 64 x 64, 3 stages (96 KB)
//   3: 256 x 256, 8 waves (4 x 2) of 64 x 128, 2 stages (128 KB)
template <int CFG> struct Cfg;
template <> struct Cfg<0> { static constexpr int TM = 2, TN = 3, WM = 4, WN = 2, NST = 2; };
template <> struct Cfg<1> { static constexpr int TM = 2, TN = 2, WM = 4, WN = 2, NST = 3; };
template <> struct Cfg<2> { static constexpr int TM = 2, TN = 2, WM = 2, WN = 2, NST = 3; };
template <> struct Cfg<3> { static constexpr int TM = 2, TN = 4, WM = 4, WN = 2, NST = 2; };
constexpr int kNumCfg = 4;

template <int CFG, bool TA, bool TB, int EPI, bool CS>
hipError_t launch_cfg(GemmArgs& a, int splits, hipStream_t st) {
  using C = Cfg<CFG>;
  constexpr int BM = C::WM * C::TM * 32, BN = C::WN * C::TN * 32;
  a.mtiles = (a.M + BM - 1) / BM;
  a.ntiles = (a.N + BN - 1) / BN;
  const int grid = splits * a.mtiles * a.ntiles;
  hipLaunchKernelGGL((k_gemm<C::TM, C::TN, C::WM, C::WN, C::NST, TA, TB, EPI, CS>), dim3(grid),
                     dim3(64 * C::WM * C::WN), 0, st, a);
  return hipGetLastError();
}

template <bool TA, bool TB, int EPI, bool CS>
hipError_t launch_any(int cfg, GemmArgs& a, int splits, hipStream_t st) {
  switch (cfg) {
    case 0: return launch_cfg<0, TA, TB, EPI, CS>(a, splits, st);
    case 1: return launch_cfg<1, TA, TB, EPI, CS>(a, splits, st);
    case 2: return launch_cfg<2, TA, TB, EPI, CS>(a, splits, st);
    default: return launch_cfg<3, TA, TB, EPI, CS>(a, splits, st);
  }
}

}  // namespace

extern "C" {

int pde_gemm_num_cfgs() { return kNumCfg; }

void pde_gemm_tile(int cfg, int* bm, int* bn) {
  static const int t[kNumCfg][2] = {{256, 192}, {256, 128}, {128, 128}, {256, 256}};
  cfg = cfg < 0 || cfg >= kNumCfg ? 0 : cfg;
  *bm = t[cfg][0];
  *bn = t[cfg][1];
}

// See the file header for the operand conventions.  epi: 0 bf16 (+bias), 1 bias+GELU (C = pre,
// C2 = act), 2 GELU backward (aux = pre), 3 fp32 split-K slabs (C = float [splits][M][ldc]).
// colsum (wgrad only): fp32 [splits][M] bias-gradient partials.  Supported combinations:
// (ta, tb) = (0, 0) with epi 0/1, (0, 1) with epi 0/2, (1, 1) with epi 0/3 (+colsum).
hipError_t pde_gemm(const void* A, const void* B, void* C, void* C2, const void* bias, const void* aux, float* colsum,
                    int ta, int tb, int epi, int M, int N, int K, int lda, int ldb, int ldc, int splits, int cfg,
                    hipStream_t st) {
  // a K-contiguous operand is staged in 8-element chunks: K % 8 == 0 unless both operands are transposed
  if (M <= 0 || N <= 0 || K <= 0 || (K % 8 && !(ta && tb)) || N % 8 || lda % 8 || ldb % 8 || ldc % 8 ||
      splits < 1)
    return hipErrorInvalidValue;
  if ((ta && M % 8) || cfg < 0 || cfg >= kNumCfg) return hipErrorInvalidValue;
  if (splits > 1 && epi != kSlab) return hipErrorInvalidValue;
  if (colsum && !(ta && tb)) return hipErrorInvalidValue;
  const size_t a_bytes = (size_t)(ta ? K : M) * lda * 2, b_bytes = (size_t)(tb ? K : N) * ldb * 2;
  if (a_bytes >= kOOB || b_bytes >= kOOB) return hipErrorInvalidValue;   // 32-bit buffer offsets
  GemmArgs a{};
  a.A = (const bf16_t*)A;
  a.B = (const bf16_t*)B;
  a.C = C;
  a.C2 = (bf16_t*)C2;
  a.bias = (const bf16_t*)bias;
  a.aux = (const bf16_t*)aux;
  a.colsum = colsum;
  a.a_bytes = (uint32_t)a_bytes;
  a.b_bytes = (uint32_t)b_bytes;
  a.M = M; a.N = N; a.K = K; a.lda = lda; a.ldb = ldb; a.ldc = ldc;
  a.kper = (((K + 63) / 64 + splits - 1) / splits) * 64;
  splits = (K + a.kper - 1) / a.kper;
  if (!ta && !tb) {
    if (epi == kBf16) return launch_any<false, false, kBf16, false>(cfg, a, splits, st);
    if (epi == kGelu) return launch_any<false, false, kGelu, false>(cfg, a, splits, st);
  } else if (!ta && tb) {
    if (epi == kBf16) return launch_any<false, true, kBf16, false>(cfg, a, splits, st);
    if (epi == kGeluBwd) return launch_any<false, true, kGeluBwd, false>(cfg, a, splits, st);
  } else if (ta && tb) {
    if (epi == kSlab) {
      return colsum ? launch_any<true, true, kSlab, true>(cfg, a, splits, st)
                    : launch_any<true, true, kSlab, false>(cfg, a, splits, st);
    }
    if (epi == kBf16) {
      return colsum ? launch_any<true, true, kBf16, true>(cfg, a, splits, st)
                    : launch_any<true, true, kBf16, false>(cfg, a, splits, st);
    }
  }
  return hipErrorInvalidValue;
}

// the number of K slices pde_gemm actually launches for a requested split count
int pde_gemm_splits(int K, int splits) {
  if (K <= 0 || splits < 1) return 1;
  const int kper = (((K + 63) / 64 + splits - 1) / splits) * 64;
  return (K + kper - 1) / kper;
}

hipError_t pde_gemm_reduce(const float* part, int S, int M, int N, void* dw, const float* cs, void* db,
                           hipStream_t st) {
  const int64_t mn = (int64_t)M * N;
  if (mn % 4 || S < 1 || (cs == nullptr) != (db == nullptr) || (part == nullptr) != (dw == nullptr))
    return hipErrorInvalidValue;
  const int nb_main = part ? (int)((mn / 4 + 255) / 256) : 0;     // part == null: fold db only
  if (nb_main == 0 && !cs) return hipSuccess;
  const int nb_db = cs ? (M + 255) / 256 : 0;
  hipLaunchKernelGGL(k_gemm_reduce, dim3(nb_main + nb_db), dim3(256), 0, st, part, S, mn, (bf16_t*)dw, nb_main, cs, M,
                     (bf16_t*)db);
  return hipGetLastError();
}

}  // extern "C"
